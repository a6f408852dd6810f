// credit2: the runqueue-per-socket credit scheduler (S4), on the GPU topology.
//
// Behaviour parity with X:xen/common/sched_credit2.c (Xen 4.2):
//   * one runqueue per "socket" -- here per GPU: every XCD partition of a GPU
//     pulls from the same credit-sorted queue (runq_insert :313-357);
//   * credit burns at max_weight/weight ns per ns of run time (t2c/c2t
//     :272-280, burn_credits :623-648), so weight shapes the share;
//   * the candidate is the highest-credit queued slot, a slot last run on
//     another partition only if it leads by the migrate resistance
//     (runq_candidate :1540-1578);
//   * when the chosen slot's credit is exhausted, every slot of the runqueue
//     gets CREDIT_INIT on top of its (clipped) carry-over (reset_credit
//     :578-621), then load is balanced across runqueues (balance_load);
//   * the run time is the credit lead over the next queued slot, clamped to
//     [MIN_TIMER, MAX_TIMER] (csched_runtime :1497-1535);
//   * a waking slot tickles its own partition if it out-credits the current
//     slot, else an idle untickled partition, else the lowest-credit one if
//     it leads it by the migrate resistance (runq_tickle :474-576);
//   * new slots go to the least-loaded runqueue their affinity allows
//     (choose_cpu).
// Credit2 has no cap and no global tslice/ratelimit in this Xen version.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <list>
#include <map>
#include <set>

#include "engine.h"

namespace gpbs {
namespace {

constexpr int64_t kUs = 1000;
constexpr int64_t kMinTimer = 500 * kUs;          // CSCHED_MIN_TIMER
constexpr int64_t kMaxTimer = 2000 * kUs;         // CSCHED_MAX_TIMER
constexpr int64_t kCreditInit = 10000 * kUs;      // CSCHED_CREDIT_INIT
constexpr int64_t kCarryoverMax = kMinTimer;      // CSCHED_CARRYOVER_MAX
constexpr int64_t kMigrateResist = 500 * kUs;     // opt_migrate_resist
constexpr int64_t kCreditReset = 0;               // CSCHED_CREDIT_RESET
constexpr int64_t kIdleCredit = -(int64_t(1) << 30);  // CSCHED_IDLE_CREDIT
constexpr int kDefaultWeight = 256;

std::string cfmt(const char* f, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}

struct C2Slot : SchedSlotData {
  int64_t credit = kCreditInit;
  int64_t start_time = 0;
  int rq = -1;  // runqueue the slot is assigned to (rqd)
  bool on_runq = false;
  uint64_t resets = 0;
};
struct C2Dom : SchedTenantData {
  int weight = kDefaultWeight;
};
struct C2Pcpu : SchedPartData {
  int rq = -1;
};
struct RunQ {
  int id = -1;
  Mask active, idle, tickled;
  std::list<int> runq;   // queued slot ids, credit-descending
  std::set<int> members; // slots assigned to this runqueue (rqd->svc)
  int max_weight = 1;
  uint64_t resets = 0, balances = 0;
};

class Credit2Scheduler : public Scheduler {
 public:
  Credit2Scheduler(Engine& e, int pool) : Scheduler(e, pool) {}
  const char* name() const override { return "SMP Credit Scheduler rev2 (credit2)"; }
  const char* opt_name() const override { return "credit2"; }

  C2Slot& sv(Slot& v) { return *static_cast<C2Slot*>(v.priv.get()); }
  C2Dom& sd(Tenant& d) { return *static_cast<C2Dom*>(d.priv.get()); }
  C2Pcpu& pc(int c) { return *static_cast<C2Pcpu*>(E.parts[c]->priv.get()); }
  int weight_of(Slot& v) {
    Tenant* t = E.tenant(v.tenant);
    return t && t->priv ? sd(*t).weight : kDefaultWeight;
  }
  RunQ* rq_of_cpu(int c) {
    if (c < 0 || c >= (int)E.parts.size() || !E.parts[c]->priv) return nullptr;
    auto it = rqs_.find(pc(c).rq);
    return it == rqs_.end() ? nullptr : &it->second;
  }

  // ----------------------------------------------------------- credits ---
  int64_t t2c(const RunQ& rq, int64_t t, Slot& v) { return t * rq.max_weight / std::max(1, weight_of(v)); }
  int64_t c2t(const RunQ& rq, int64_t c, Slot& v) { return c * weight_of(v) / std::max(1, rq.max_weight); }

  void burn(RunQ& rq, Slot& v, int64_t now) {
    if (v.is_idle()) return;
    C2Slot& s = sv(v);
    const int64_t dt = now - s.start_time;
    if (dt <= 0) return;
    s.credit -= t2c(rq, dt, v);
    s.start_time = now;
  }

  void update_max_weight(RunQ& rq) {
    int mw = 1;
    for (int sid : rq.members) mw = std::max(mw, weight_of(*E.slots[sid]));
    rq.max_weight = mw;
  }

  void assign(Slot& v, int rqid) {
    C2Slot& s = sv(v);
    if (s.rq == rqid) return;
    if (s.on_runq) runq_remove(v);
    if (auto it = rqs_.find(s.rq); it != rqs_.end()) {
      it->second.members.erase(v.id);
      update_max_weight(it->second);
    }
    s.rq = rqid;
    if (auto it = rqs_.find(rqid); it != rqs_.end()) {
      it->second.members.insert(v.id);
      update_max_weight(it->second);
    }
  }

  void runq_insert(RunQ& rq, Slot& v) {
    C2Slot& s = sv(v);
    auto it = rq.runq.begin();
    for (; it != rq.runq.end(); ++it)
      if (s.credit > sv(*E.slots[*it]).credit) break;
    rq.runq.insert(it, v.id);
    s.on_runq = true;
  }
  void runq_remove(Slot& v) {
    C2Slot& s = sv(v);
    if (!s.on_runq) return;
    if (auto it = rqs_.find(s.rq); it != rqs_.end()) it->second.runq.remove(v.id);
    s.on_runq = false;
  }

  void reset_credit(RunQ& rq, int64_t now) {
    for (int sid : rq.members) {
      C2Slot& s = sv(*E.slots[sid]);
      if (s.credit > kCarryoverMax) s.credit = kCarryoverMax;
      s.credit += kCreditInit;
      s.start_time = now;
      s.resets++;
    }
    rq.resets++;
    // Clipping can reorder the queue; keep it sorted.
    rq.runq.sort([&](int a, int b) { return sv(*E.slots[a]).credit > sv(*E.slots[b]).credit; });
    E.emit(TRC_ACCT, 0, (uint32_t)pool_, (uint32_t)rq.members.size(), 0, (uint32_t)rq.id);
  }

  int load(RunQ& rq) {
    int n = 0;
    for (int sid : rq.members) {
      Slot& v = *E.slots[sid];
      if (E.runnable(v) && (sv(v).on_runq || v.is_running)) n++;
    }
    return n;
  }

  // balance_load: move one queued slot from this runqueue to the least
  // loaded one when the imbalance is at least two runnable slots.
  void balance_load(RunQ& rq, int64_t now) {
    RunQ* best = nullptr;
    int bl = 1 << 30;
    for (auto& kv : rqs_) {
      if (&kv.second == &rq || kv.second.active.empty()) continue;
      const int l = load(kv.second);
      if (l < bl) {
        bl = l;
        best = &kv.second;
      }
    }
    if (!best || load(rq) - bl < 2) return;
    for (auto it = rq.runq.rbegin(); it != rq.runq.rend(); ++it) {  // lowest credit first
      Slot& v = *E.slots[*it];
      const Mask ok = best->active & v.affinity;
      if (ok.empty()) continue;
      runq_remove(v);
      assign(v, best->id);
      const Mask idle = ok & best->idle;
      v.processor = idle.empty() ? ok.first() : idle.first();
      sv(v).start_time = now;
      runq_insert(*best, v);
      tickle(*best, v.processor, v, now);
      best->balances++;
      E.perfc.incr(PC_migrate_queued);
      return;
    }
  }

  void tickle(RunQ& rq, int cpu, Slot& nv, int64_t now) {
    const Mask aff = nv.affinity & rq.active;
    int ipid = -1;
    Slot& cur = E.curr_of(cpu);
    burn(rq, cur, now);
    const int64_t cur_credit = cur.is_idle() ? kIdleCredit : sv(cur).credit;
    if (aff.test(cpu) && cur_credit < sv(nv).credit) {
      ipid = cpu;
    } else {
      const Mask idle = (rq.idle & aff).andnot(rq.tickled);
      if (!idle.empty()) {
        ipid = idle.first();
      } else {
        int64_t lowest = int64_t(1) << 62;
        const Mask busy = aff.andnot(rq.idle).andnot(rq.tickled);
        for (int c = busy.first(); c >= 0; c = busy.next(c + 1)) {
          if (c == cpu) continue;
          Slot& o = E.curr_of(c);
          if (o.is_idle()) continue;
          burn(rq, o, now);
          if (sv(o).credit < lowest) {
            lowest = sv(o).credit;
            ipid = c;
          }
        }
        if (ipid >= 0 && lowest + kMigrateResist > sv(nv).credit) ipid = -1;
      }
    }
    if (ipid < 0) {
      E.perfc.incr(PC_tickle_idlers_none);
      return;
    }
    rq.tickled.set(ipid);
    E.perfc.incr(PC_tickle_idlers_some);
    E.raise_softirq(ipid);
  }

  // ----------------------------------------------------------- hooks ----
  void alloc_pdata(int cpu) override {
    E.parts[cpu]->priv = std::make_unique<C2Pcpu>();
    const int id = E.parts[cpu]->gpu;
    RunQ& rq = rqs_[id];
    rq.id = id;
    rq.active.set(cpu);
    rq.idle.set(cpu);
    pc(cpu).rq = id;
  }
  void free_pdata(int cpu) override {
    if (RunQ* rq = rq_of_cpu(cpu)) {
      rq->active.clear(cpu);
      rq->idle.clear(cpu);
      rq->tickled.clear(cpu);
      if (rq->active.empty()) {  // deactivate: its slots get reassigned on wake
        for (int sid : std::vector<int>(rq->members.begin(), rq->members.end())) {
          Slot& v = *E.slots[sid];
          runq_remove(v);
          sv(v).rq = -1;
        }
        rqs_.erase(rq->id);
      }
    }
    E.parts[cpu]->priv.reset();
  }
  int init_domain(Tenant& d) override {
    d.priv = std::make_unique<C2Dom>();
    return 0;
  }
  void destroy_domain(Tenant& d) override { d.priv.reset(); }
  void alloc_vdata(Slot& v) override {
    v.priv = std::make_unique<C2Slot>();
    if (v.is_idle()) sv(v).credit = kIdleCredit;
  }
  void insert_vcpu(Slot& v) override {
    if (v.is_idle()) return;
    if (RunQ* rq = rq_of_cpu(v.processor)) assign(v, rq->id);
    sv(v).start_time = E.now();
  }
  void remove_vcpu(Slot& v) override {
    runq_remove(v);
    if (auto it = rqs_.find(sv(v).rq); it != rqs_.end()) {
      it->second.members.erase(v.id);
      update_max_weight(it->second);
    }
    sv(v).rq = -1;
  }
  void sleep(Slot& v) override {
    E.perfc.incr(PC_vcpu_sleep);
    if (E.parts[v.processor]->curr == v.id)
      E.raise_softirq(v.processor);
    else
      runq_remove(v);
  }
  void wake(Slot& v) override {
    if (E.parts[v.processor]->curr == v.id) {
      E.perfc.incr(PC_vcpu_wake_running);
      return;
    }
    if (sv(v).on_runq) {
      E.perfc.incr(PC_vcpu_wake_onrunq);
      return;
    }
    E.perfc.incr(PC_vcpu_wake_runnable);
    RunQ* rq = rq_of_cpu(v.processor);
    if (!rq || !v.affinity.test(v.processor)) {
      v.processor = pick_cpu(v);
      rq = rq_of_cpu(v.processor);
      if (!rq) return;
    }
    assign(v, rq->id);
    const int64_t now = E.now();
    sv(v).start_time = now;
    runq_insert(*rq, v);
    tickle(*rq, v.processor, v, now);
  }
  void yield(Slot&) override {}  // credit2 (4.2) has no yield handling beyond rescheduling

  int pick_cpu(Slot& v) override {
    RunQ* best = nullptr;
    int bl = 1 << 30;
    RunQ* own = rq_of_cpu(v.processor);
    for (auto& kv : rqs_) {
      RunQ& rq = kv.second;
      if ((rq.active & v.affinity).empty()) continue;
      int l = load(rq) - (sv(v).rq == rq.id && E.runnable(v) ? 1 : 0);
      if (l < bl || (l == bl && &rq == own)) {
        bl = l;
        best = &rq;
      }
    }
    const Mask pool = E.pools[pool_]->cpus;
    if (!best) return pool.test(v.processor) ? v.processor : pool.first();
    const Mask ok = best->active & v.affinity;
    if (ok.test(v.processor)) return v.processor;
    const Mask idle = ok & best->idle;
    return idle.empty() ? ok.first() : idle.first();
  }

  Slot* candidate(RunQ& rq, Slot& scurr, int cpu) {
    Slot* snext = (!scurr.is_idle() && E.runnable(scurr) && scurr.affinity.test(cpu))
                      ? &scurr
                      : E.slots[E.parts[cpu]->idle_slot].get();
    const int64_t cc = snext->is_idle() ? kIdleCredit : sv(*snext).credit;
    for (int sid : rq.runq) {
      Slot& s = *E.slots[sid];
      if (!s.affinity.test(cpu)) continue;
      if (s.processor != cpu && cc + kMigrateResist > sv(s).credit) continue;
      if (sv(s).credit > cc) snext = &s;
      break;
    }
    return snext;
  }

  TaskSlice do_schedule(int cpu, int64_t now) override {
    E.perfc.incr(PC_schedule);
    Slot& scurr = E.curr_of(cpu);
    RunQ* rqp = rq_of_cpu(cpu);
    if (!rqp) return TaskSlice{E.parts[cpu]->idle_slot, -1, false};
    RunQ& rq = *rqp;
    rq.tickled.clear(cpu);
    burn(rq, scurr, now);
    Slot* snext = candidate(rq, scurr, cpu);
    if (snext != &scurr && !scurr.is_idle() && E.runnable(scurr) && !sv(scurr).on_runq) {
      if (sv(scurr).rq != rq.id) assign(scurr, rq.id);
      runq_insert(rq, scurr);
    }
    TaskSlice ret{snext->id, -1, false};
    if (!snext->is_idle()) {
      if (snext != &scurr) {
        runq_remove(*snext);
        if (snext->processor != cpu) {
          snext->processor = cpu;
          ret.migrated = true;
        }
      }
      if (sv(*snext).credit <= kCreditReset) {
        reset_credit(rq, now);
        balance_load(rq, now);
      }
      sv(*snext).start_time = now;
      rq.idle.clear(cpu);
      // csched_runtime: the lead over the next queued slot, clamped.
      int64_t t = c2t(rq, sv(*snext).credit, *snext);
      if (!rq.runq.empty()) {
        Slot& nx = *E.slots[rq.runq.front()];
        const int64_t nt = c2t(rq, sv(*snext).credit - sv(nx).credit, *snext);
        t = std::min(t, nt);
      }
      ret.time_ns = std::clamp(t, kMinTimer, kMaxTimer);
    } else {
      rq.idle.set(cpu);
    }
    return ret;
  }

  int adjust(Tenant& d, bool set, int* weight, int* cap) override {
    C2Dom& s = sd(d);
    if (set) {
      if (*weight != -1 && *weight != 0) {
        if (*weight < 1 || *weight > GPBS_WEIGHT_MAX) return GPBS_ERANGE;
        s.weight = *weight;
        for (auto& kv : rqs_) update_max_weight(kv.second);
      }
    }
    *weight = s.weight;
    *cap = 0;  // credit2 has no caps
    return GPBS_OK;
  }
  int adjust_ext(Tenant& d, bool set, gpbs_sched_ext_t& x) override {
    int w = set ? x.weight : -1, c = -1;
    int rc = adjust(d, set, &w, &c);
    if (rc) return rc;
    x = gpbs_sched_ext_t{};
    x.weight = w;
    int64_t cr = 0;
    for (int sid : d.slots) cr += sv(*E.slots[sid]).credit;
    x.credit = d.slots.empty() ? 0 : (int32_t)(cr / (int64_t)d.slots.size() / kUs);
    return GPBS_OK;
  }
  int adjust_global(bool set, int* tslice_us, int* ratelimit_us) override {
    if (set) return GPBS_EINVAL;  // no global parameters (sched_adjust_global unsupported)
    *tslice_us = (int)(kMaxTimer / kUs);
    *ratelimit_us = 0;
    return GPBS_OK;
  }
  uint32_t trace_word(Slot& v) override {
    if (!v.priv) return 0;
    const int64_t c = v.is_idle() ? 0 : std::clamp<int64_t>(sv(v).credit / kUs, -(1 << 23), (1 << 23) - 1);
    return (uint32_t)128 | ((uint32_t)c << 8);
  }
  void fill_tenant_info(Tenant& d, gpbs_tenant_info_t& o) override {
    o.weight = sd(d).weight;
    o.cap = 0;
    o.tslice_us = (uint32_t)(kMaxTimer / kUs);
    o.tick_period_us = 0;
    int active = 0;
    for (int sid : d.slots) active += E.runnable(*E.slots[sid]);
    o.active_slots = active;
  }
  void fill_slot_info(Slot& v, gpbs_slot_info_t& o) override {
    o.credit = (int32_t)std::clamp<int64_t>(sv(v).credit / kUs, INT32_MIN, INT32_MAX);
    o.on_runq = sv(v).on_runq;
    o.pri = 0;
  }
  void dump_settings(std::string& o) override {
    o += cfmt("Scheduler: %s\nActive queues: %zu\n\tdefault-weight     = %d\n", name(), rqs_.size(),
              kDefaultWeight);
    for (auto& kv : rqs_) {
      RunQ& rq = kv.second;
      o += cfmt("Runqueue %d:\n\tncpus              = %d\n\tmax_weight         = %d\n\tinstload           = %d\n"
                "\tresets             = %llu\n\tbalances           = %llu\n",
                rq.id, rq.active.weight(), rq.max_weight, load(rq), (unsigned long long)rq.resets,
                (unsigned long long)rq.balances);
    }
  }
  void dump_cpu_state(int cpu, std::string& o) override {
    RunQ* rq = rq_of_cpu(cpu);
    o += cfmt(" runqueue %d\n", rq ? rq->id : -1);
    Slot& c = E.curr_of(cpu);
    if (!c.is_idle()) o += cfmt("\trun: [%d.%d] credit=%lld\n", c.tenant, c.index, (long long)(sv(c).credit / kUs));
    if (!rq) return;
    int n = 0;
    for (int sid : rq->runq) {
      Slot& v = *E.slots[sid];
      if (v.processor != cpu) continue;
      o += cfmt("\t%3d: [%d.%d] credit=%lld\n", ++n, v.tenant, v.index, (long long)(sv(v).credit / kUs));
    }
  }
  void dump_admin_conf(std::string& o) override {
    for (auto& tp : E.tenants) {
      if (!tp || !tp->alive || tp->pool != pool_ || !tp->priv) continue;
      o += cfmt("dom%d weight=%d credits(us):", tp->id, sd(*tp).weight);
      for (int sid : tp->slots) o += cfmt(" %lld", (long long)(sv(*E.slots[sid]).credit / kUs));
      o += "\n";
    }
  }
  std::string check() override {
    for (auto& kv : rqs_) {
      RunQ& rq = kv.second;
      int64_t prev = INT64_MAX;
      for (int sid : rq.runq) {
        Slot& v = *E.slots[sid];
        if (!sv(v).on_runq || sv(v).rq != rq.id) return cfmt("credit2: slot %d queued on rq %d inconsistently", sid, rq.id);
        if (v.is_running) return cfmt("credit2: running slot %d on runq", sid);
        if (!rq.members.count(sid)) return cfmt("credit2: queued slot %d not a member of rq %d", sid, rq.id);
        (void)prev;
      }
    }
    return "";
  }

 private:
  std::map<int, RunQ> rqs_;
};

}  // namespace

std::unique_ptr<Scheduler> make_credit2_scheduler(Engine& e, int pool) {
  return std::make_unique<Credit2Scheduler>(e, pool);
}

}  // namespace gpbs
