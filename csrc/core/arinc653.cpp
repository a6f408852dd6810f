// ARINC 653 time-partition scheduler (S4; X:xen/common/sched_arinc653.c).
//
// A fixed cyclic schedule: a major frame divided into windows, each window
// owned by one tenant (or by one slot of it), repeated forever.  Inside a
// window only the owner runs; when the owner has nothing runnable the
// partitions idle -- temporal isolation, never work-conserving.  The
// schedule is installed through the control API (gpbs_arinc653_set, the
// XEN_SYSCTL_SCHEDOP_putinfo of a653sched_adjust_global) and takes effect
// at once: a new major frame starts at the next dispatch (:282-285).
//
// GPU-native shape: the reference runs on ONE pCPU (a653sched_pick_cpu
// returns 0).  Here a pool spans many partitions (XCDs / shader engines of
// one or more GPUs); every partition of the pool follows the SAME window
// table on the same clock, so a window hands the whole pool to its tenant
// and all partitions switch together (gang-aligned time partitioning).  An
// entry naming a slot (slot >= 0) runs just that slot on its own partition,
// the rest idle -- the reference's per-vCPU entries; slot -1 runs every slot
// of the tenant, slot k on pool partition k mod n.
//
// Deliberate differences (SURVEY §7.6 style):
//  * Q15: the schedule need not contain a Domain-0 entry (the reference
//    rejects one without dom0, :237-258) -- Domain-0 here is the control
//    plane's placeholder tenant, not the toolstack that must stay alive.
//  * Q16: until a schedule is installed the pool runs an automatic one --
//    every live tenant one window of tslice_us (default 10 ms) in creation
//    order -- instead of the reference's dom0-only 10 ms frame (:347-356),
//    which would run nothing else until a toolstack put a table.
//  * Window position is derived from (now - frame start) on every call, not
//    the reference's function-static sched_index shared by all CPUs
//    (:520-525), which is only correct on one pCPU.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <vector>

#include "engine.h"

namespace gpbs {
namespace {

std::string afmt(const char* f, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}

struct ASlot : SchedSlotData {
  bool awake = false;
};
struct ADom : SchedTenantData {
  int weight = 256;
};
struct APcpu : SchedPartData {};

using Entry = ArincEntry;

class Arinc653Scheduler : public Scheduler {
 public:
  Arinc653Scheduler(Engine& e, int pool) : Scheduler(e, pool) {}
  const char* name() const override { return "ARINC 653 Scheduler (time partitions)"; }
  const char* opt_name() const override { return "arinc653"; }

  int init() override {
    auto_slice_ns_ = (int64_t)kDefaultWindowUs * 1000;
    return 0;
  }
  ASlot& sv(Slot& v) { return *static_cast<ASlot*>(v.priv.get()); }
  Mask cpus() { return E.pools[pool_]->cpus; }

  // ------------------------------------------------------ schedule table --
  int set_schedule(int64_t major_ns, const std::vector<Entry>& es) override {
    if (major_ns <= 0 || es.empty() || es.size() > (size_t)GPBS_ARINC653_MAX_ENTRIES) return GPBS_EINVAL;
    int64_t total = 0;
    for (const Entry& x : es) {
      if (x.runtime <= 0 || x.slot < -1 || x.slot >= kMaxSlotIndex) return GPBS_EINVAL;
      total += x.runtime;
    }
    if (total > major_ns) return GPBS_EINVAL;  // frame too short for its windows (:260-262)
    table_ = es;
    major_ns_ = major_ns;
    explicit_ = true;
    next_major_ = E.now();  // effective at once (:282-285)
    kick_all();
    return 0;
  }
  int get_schedule(int64_t* major_ns, std::vector<Entry>* es) override {
    refresh_auto();
    *major_ns = major_ns_;
    *es = table_;
    return explicit_ ? 1 : 0;
  }

  // Q16 automatic table: one tslice window per live tenant, creation order.
  void refresh_auto() {
    if (explicit_) return;
    std::vector<Entry> es;
    for (auto& t : E.tenants)
      if (t && t->alive && t->pool == pool_ && t->priv && t->name != "Domain-0")
        es.push_back(Entry{t->id, -1, auto_slice_ns_});
    if (es.empty()) es.push_back(Entry{-1, -1, auto_slice_ns_});  // idle frame
    if (es.size() != table_.size() || !std::equal(es.begin(), es.end(), table_.begin(), [](const Entry& a, const Entry& b) {
          return a.tenant == b.tenant && a.slot == b.slot && a.runtime == b.runtime;
        })) {
      table_ = es;
      major_ns_ = 0;
      for (const Entry& x : es) major_ns_ += x.runtime;
      next_major_ = E.now();
    }
  }

  void kick_all() {
    Mask m = cpus();
    for (int c = m.first(); c >= 0; c = m.next(c + 1)) E.raise_softirq(c);
  }

  // ------------------------------------------------------------- hooks ---
  void alloc_pdata(int cpu) override { E.parts[cpu]->priv = std::make_unique<APcpu>(); }
  void free_pdata(int cpu) override { E.parts[cpu]->priv.reset(); }
  int init_domain(Tenant& d) override {
    d.priv = std::make_unique<ADom>();
    return 0;
  }
  void destroy_domain(Tenant& d) override {
    d.priv.reset();
    if (!explicit_) kick_all();
  }
  void alloc_vdata(Slot& v) override { v.priv = std::make_unique<ASlot>(); }
  void insert_vcpu(Slot& v) override {
    sv(v).awake = E.runnable(v);
    if (!explicit_) kick_all();
  }
  void remove_vcpu(Slot& v) override { sv(v).awake = false; }
  void sleep(Slot& v) override {
    sv(v).awake = false;
    if (E.parts[v.processor]->curr == v.id) E.raise_softirq(v.processor);
  }
  void wake(Slot& v) override {  // a653sched_vcpu_wake
    sv(v).awake = true;
    E.raise_softirq(v.processor);
  }
  void yield(Slot&) override {}

  // Slot k of a tenant lives on pool partition k mod n (no migration, :606-611).
  int pick_cpu(Slot& v) override {
    std::vector<int> cs;
    Mask m = cpus();
    for (int c = m.first(); c >= 0; c = m.next(c + 1)) cs.push_back(c);
    if (cs.empty()) return v.processor;
    return cs[(size_t)v.index % cs.size()];
  }

  // a653sched_do_schedule (:516-597), on the pool's shared frame clock.
  TaskSlice do_schedule(int cpu, int64_t now) override {
    refresh_auto();
    if (now >= next_major_) {  // enter a new major frame
      frame_start_ = now;
      next_major_ = now + major_ns_;
      frames_++;
    }
    int64_t end = frame_start_;
    int idx = -1;
    for (size_t i = 0; i < table_.size(); ++i) {
      end += table_[i].runtime;
      if (now < end) {
        idx = (int)i;
        break;
      }
    }
    int64_t switch_at = idx >= 0 ? end : next_major_;  // past the last window: idle to the frame end
    const int idle = E.parts[cpu]->idle_slot;
    int pick = idle;
    if (idx >= 0 && table_[idx].tenant >= 0) {
      Tenant* t = E.tenant(table_[idx].tenant);
      if (t && t->alive && t->pool == pool_) {
        for (int sid : t->slots) {
          Slot& v = *E.slots[sid];
          if (table_[idx].slot >= 0 && v.index != table_[idx].slot) continue;
          if (v.processor != cpu || !sv(v).awake || !E.runnable(v)) continue;
          pick = v.id;
          break;
        }
      }
    }
    if (switch_at <= now) switch_at = now + 1000;  // never a zero-length slice
    return TaskSlice{pick, switch_at - now, false};
  }

  int adjust(Tenant& d, bool set, int* weight, int* cap) override {
    ADom& s = *static_cast<ADom*>(d.priv.get());
    if (!set) {
      *weight = s.weight;
      *cap = 0;
      return 0;
    }
    if (*weight != -1 && *weight != 0) {
      if (*weight < 1 || *weight > GPBS_WEIGHT_MAX) return GPBS_ERANGE;
      s.weight = *weight;  // recorded; the cyclic table alone decides time
    }
    return 0;
  }
  // The pool "tslice" is the automatic table's window length.
  int adjust_global(bool set, int* tslice_us, int* ratelimit_us) override {
    if (set) {
      if (*tslice_us < GPBS_TSLICE_UMIN || *tslice_us > GPBS_TSLICE_UMAX) return GPBS_EINVAL;
      auto_slice_ns_ = (int64_t)*tslice_us * 1000;
      if (!explicit_) table_.clear();
    }
    *tslice_us = (int)(auto_slice_ns_ / 1000);
    *ratelimit_us = 0;
    return 0;
  }
  void fill_tenant_info(Tenant& d, gpbs_tenant_info_t& o) override {
    int64_t w = 0;
    for (const Entry& x : table_)
      if (x.tenant == d.id) w += x.runtime;
    o.tslice_us = (int)(w / 1000);  // this tenant's time per major frame
    o.weight = static_cast<ADom*>(d.priv.get())->weight;
  }
  void fill_slot_info(Slot& v, gpbs_slot_info_t& o) override { o.on_runq = sv(v).awake; }
  void dump_settings(std::string& o) override {
    refresh_auto();
    o += afmt("arinc653: major_frame=%lldus entries=%zu%s frames=%llu\n", (long long)(major_ns_ / 1000),
              table_.size(), explicit_ ? "" : " (automatic)", (unsigned long long)frames_);
  }
  void dump_cpu_state(int cpu, std::string& o) override { o += afmt(" cpu%d\n", cpu); }
  void dump_admin_conf(std::string& o) override {
    refresh_auto();
    int64_t at = 0;
    for (const Entry& x : table_) {
      o += afmt("  window [%8lld, %8lld) us: dom%d slot %s\n", (long long)(at / 1000),
                (long long)((at + x.runtime) / 1000), x.tenant, x.slot < 0 ? "all" : std::to_string(x.slot).c_str());
      at += x.runtime;
    }
    if (at < major_ns_)
      o += afmt("  window [%8lld, %8lld) us: idle\n", (long long)(at / 1000), (long long)(major_ns_ / 1000));
  }

 private:
  static constexpr int kDefaultWindowUs = 10000;  // MILLISECS(10), :352-355
  static constexpr int kMaxSlotIndex = 4096;      // MAX_VIRT_CPUS analog (:243)
  std::vector<Entry> table_;
  int64_t major_ns_ = 0, frame_start_ = 0, next_major_ = 0, auto_slice_ns_ = 0;
  uint64_t frames_ = 0;
  bool explicit_ = false;
};

}  // namespace

std::unique_ptr<Scheduler> make_arinc653_scheduler(Engine& e, int pool) {
  return std::make_unique<Arinc653Scheduler>(e, pool);
}

}  // namespace gpbs
