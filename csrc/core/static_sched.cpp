// Static partition scheduler: the ARINC-653 analog (X:xen/common/sched_arinc653.c,
// static cyclic partitions) used as the "static equal XCD split" baseline policy.
// Partitions of the pool are divided among live tenants in proportion to their
// weights (largest remainder); a partition only ever runs slots of its owner,
// round-robin with the pool quantum; when the owner has nothing runnable the
// partition idles (non work-conserving, like a static CU mask).
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <list>
#include <map>

#include "engine.h"

namespace gpbs {
namespace {

std::string sfmt(const char* f, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}

struct SSlot : SchedSlotData {
  int runq_cpu = -1;
};
struct SDom : SchedTenantData {
  int weight = 256;
  int cap = 0;
};
struct SPcpu : SchedPartData {
  std::list<int> runq;
  int owner = -1;
};

class StaticScheduler : public Scheduler {
 public:
  StaticScheduler(Engine& e, int pool) : Scheduler(e, pool) {}
  const char* name() const override { return "Static partition scheduler (ARINC653-like)"; }
  const char* opt_name() const override { return "static"; }

  int init() override {
    tslice_us_ = std::max(GPBS_TSLICE_UMIN, std::min(GPBS_TSLICE_UMAX, E.boot.tslice_us));
    return 0;
  }
  SPcpu& pc(int c) { return *static_cast<SPcpu*>(E.parts[c]->priv.get()); }
  SSlot& sv(Slot& v) { return *static_cast<SSlot*>(v.priv.get()); }
  SDom& sd(Tenant& d) { return *static_cast<SDom*>(d.priv.get()); }
  Mask cpus() { return E.pools[pool_]->cpus; }

  // Recompute partition ownership and re-home every slot onto its owner's cpus.
  void rebalance() {
    std::vector<int> ts;
    for (auto& t : E.tenants)
      if (t && t->alive && t->pool == pool_ && t->priv) ts.push_back(t->id);
    std::vector<int> cs;
    Mask m = cpus();
    for (int c = m.first(); c >= 0; c = m.next(c + 1)) cs.push_back(c);
    for (int c : cs) pc(c).owner = -1;
    owned_.clear();
    if (ts.empty() || cs.empty()) return;
    long wsum = 0;
    for (int t : ts) wsum += sd(*E.tenants[t]).weight;
    std::vector<std::pair<double, int>> rem;
    std::vector<int> share(ts.size(), 0);
    int given = 0;
    for (size_t i = 0; i < ts.size(); ++i) {
      double exact = (double)cs.size() * sd(*E.tenants[ts[i]]).weight / wsum;
      share[i] = (int)exact;
      given += share[i];
      rem.push_back({exact - share[i], (int)i});
    }
    std::sort(rem.begin(), rem.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first > b.first : a.second < b.second; });
    for (size_t k = 0; given < (int)cs.size() && k < rem.size(); ++k, ++given) share[rem[k].second]++;
    // Tenants with zero share (more tenants than partitions) share round-robin.
    size_t ci = 0;
    for (size_t i = 0; i < ts.size(); ++i)
      for (int k = 0; k < share[i] && ci < cs.size(); ++k) {
        pc(cs[ci]).owner = ts[i];
        owned_[ts[i]].push_back(cs[ci++]);
      }
    for (size_t i = 0; i < ts.size(); ++i)
      if (owned_[ts[i]].empty()) owned_[ts[i]].push_back(cs[i % cs.size()]);
    for (int t : ts) {
      Tenant& d = *E.tenants[t];
      auto& own = owned_[t];
      for (size_t k = 0; k < d.slots.size(); ++k) {
        Slot& v = *E.slots[d.slots[k]];
        int target = own[k % own.size()];
        if (v.processor == target) continue;
        if (sv(v).runq_cpu >= 0) {
          pc(sv(v).runq_cpu).runq.remove(v.id);
          sv(v).runq_cpu = -1;
          v.processor = target;
          enqueue(v);
        } else if (v.is_running) {
          v.pause_flags |= VPF_MIGRATING;  // moved on deschedule
          E.raise_softirq(v.processor);
        } else {
          v.processor = target;
        }
      }
    }
    for (int c : cs) E.raise_softirq(c);
  }

  void enqueue(Slot& v) {
    pc(v.processor).runq.push_back(v.id);
    sv(v).runq_cpu = v.processor;
    E.raise_softirq(v.processor);
  }

  void alloc_pdata(int cpu) override {
    E.parts[cpu]->priv = std::make_unique<SPcpu>();
    rebalance();
  }
  void free_pdata(int cpu) override {
    for (int sid : pc(cpu).runq) sv(*E.slots[sid]).runq_cpu = -1;
    E.parts[cpu]->priv.reset();
  }
  int init_domain(Tenant& d) override {
    d.priv = std::make_unique<SDom>();
    return 0;
  }
  void destroy_domain(Tenant& d) override {
    d.priv.reset();
    owned_.erase(d.id);
    if (!cpus().empty()) rebalance();
  }
  void alloc_vdata(Slot& v) override { v.priv = std::make_unique<SSlot>(); }
  void insert_vcpu(Slot& v) override {
    if (!cpus().empty() && v.index == 0 && v.tenant >= 0) rebalance();
    if (sv(v).runq_cpu < 0 && E.runnable(v) && !v.is_running) enqueue(v);
  }
  void remove_vcpu(Slot& v) override {
    if (sv(v).runq_cpu >= 0) {
      pc(sv(v).runq_cpu).runq.remove(v.id);
      sv(v).runq_cpu = -1;
    }
  }
  void sleep(Slot& v) override {
    if (E.parts[v.processor]->curr == v.id)
      E.raise_softirq(v.processor);
    else
      remove_vcpu(v);
  }
  void wake(Slot& v) override {
    if (E.parts[v.processor]->curr == v.id || sv(v).runq_cpu >= 0) return;
    enqueue(v);
  }
  void yield(Slot&) override {}
  int pick_cpu(Slot& v) override {
    auto it = owned_.find(v.tenant);
    if (it != owned_.end() && !it->second.empty()) return it->second[v.index % it->second.size()];
    return cpus().test(v.processor) ? v.processor : cpus().first();
  }

  TaskSlice do_schedule(int cpu, int64_t) override {
    Slot& cur = E.curr_of(cpu);
    SPcpu& p = pc(cpu);
    if (!cur.is_idle() && E.runnable(cur) && cur.processor == cpu) {
      p.runq.push_back(cur.id);
      sv(cur).runq_cpu = cpu;
    }
    for (auto it = p.runq.begin(); it != p.runq.end(); ++it) {
      Slot& v = *E.slots[*it];
      if (v.tenant == p.owner || p.owner < 0) {
        p.runq.erase(it);
        sv(v).runq_cpu = -1;
        return TaskSlice{v.id, (int64_t)tslice_us_ * 1000, false};
      }
    }
    return TaskSlice{E.parts[cpu]->idle_slot, -1, false};
  }

  int adjust(Tenant& d, bool set, int* weight, int* cap) override {
    SDom& s = sd(d);
    if (!set) {
      *weight = s.weight;
      *cap = s.cap;
      return 0;
    }
    if (*weight != -1 && *weight != 0) {
      if (*weight < 1 || *weight > GPBS_WEIGHT_MAX) return GPBS_ERANGE;
      s.weight = *weight;
    }
    if (*cap != -1) s.cap = *cap;
    rebalance();
    return 0;
  }
  int adjust_global(bool set, int* tslice_us, int* ratelimit_us) override {
    if (set) {
      if (*tslice_us < GPBS_TSLICE_UMIN || *tslice_us > GPBS_TSLICE_UMAX) return GPBS_EINVAL;
      tslice_us_ = *tslice_us;
    }
    *tslice_us = tslice_us_;
    *ratelimit_us = 0;
    return 0;
  }
  void fill_tenant_info(Tenant& d, gpbs_tenant_info_t& o) override {
    o.weight = sd(d).weight;
    o.cap = sd(d).cap;
    o.tslice_us = tslice_us_;
  }
  void fill_slot_info(Slot& v, gpbs_slot_info_t& o) override { o.on_runq = sv(v).runq_cpu >= 0; }
  void dump_settings(std::string& o) override { o += sfmt("static: tslice=%dus\n", tslice_us_); }
  void dump_cpu_state(int cpu, std::string& o) override {
    o += sfmt(" owner=dom%d runq=%zu\n", pc(cpu).owner, pc(cpu).runq.size());
  }
  void dump_admin_conf(std::string& o) override {
    for (auto& kv : owned_) {
      o += sfmt("dom%d partitions:", kv.first);
      for (int c : kv.second) o += sfmt(" %d", c);
      o += "\n";
    }
  }

 private:
  int tslice_us_ = 1000;
  std::map<int, std::vector<int>> owned_;
};

}  // namespace

std::unique_ptr<Scheduler> make_static_scheduler(Engine& e, int pool) {
  return std::make_unique<StaticScheduler>(e, pool);
}

}  // namespace gpbs
