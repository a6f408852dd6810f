// Credit scheduler with the PBS per-tenant adaptive quantum.
//
// Behavior parity (X: = /root/reference/xen-4.2.1/):
//   priorities / flags           X:xen/common/sched_credit.c:62-75
//   __runq_insert / tickle       :489-525, :550-610
//   burn_credits (1 credit/us)   :527-543
//   _csched_cpu_pick             :765-852
//   vcpu_acct (+migrate)         :907-949
//   wake (BOOST) / sleep / yield :1021-1101
//   dom_cntl / sys_cntl          :1103-1174  (Q2 fix: recompute derived fields)
//   dom_init (PBS state)         :1196-1237
//   runq_sort                    :1259-1300
//   acct (+P1g ceiling)          :1302-1519
//   tick (per-tenant period)     :1521-1557
//   runq_steal / load_balance    :1559-1672
//   do_schedule (per-tenant q)   :1678-1809
//   metric tick / dom update     :391-465  (Q3/Q5 fixes)
//   dumps r / z                  :1811-1974
//   ATC policy (mode "atc")      X:xen/common/sched_credit_atc.c:462-543,1916
//
// Modes: "credit"       PBS adaptive credit (the reference's built default),
//        "credit-fixed" upstream credit (global quantum, no adaptation),
//        "credit-classq" fixed per-class quanta, no phase detector: the
//                       contention class (the same counters, EWMA and band)
//                       maps straight to the PBS bounds -- memory class
//                       max_us, compute class min_us.  The ablation that
//                       tells what the detector (:302-389) adds over a
//                       class -> quantum table,
//        "atc"          spin-latency driven global re-slicing.
#include <algorithm>
#include <cinttypes>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <list>

#include "engine.h"

namespace gpbs {

namespace {
constexpr uint16_t FLAG_PARKED = 0x1;
constexpr uint16_t FLAG_YIELD = 0x2;
constexpr int kDefaultWeight = 256;

std::string fmt(const char* f, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}

enum class Mode { PBS, FIXED, ATC, CLASSQ };

struct CSlot : SchedSlotData {
  int runq_cpu = -1;  // != -1 while on a runq (__vcpu_on_runq)
  bool active = false;
  int32_t credit = 0;
  int64_t start_time = 0;
  uint16_t flags = 0;
  int16_t pri = PRI_UNDER;
  int64_t req_until = 0;  // boost_exclusive: a BOOSTed wake's request window (ns)
  uint64_t prev_pmc[kNumPmc] = {0, 0, 0, 0};
  struct {
    int32_t credit_last = 0;
    uint32_t credit_incr = 0, state_active = 0, state_idle = 0, migrate_q = 0, migrate_r = 0;
  } stats;
};

struct CDom : SchedTenantData {
  std::list<int> active_vcpu;  // slot ids (list_add => push_front)
  bool on_active = false;
  uint16_t active_vcpu_count = 0;
  uint16_t weight = kDefaultWeight;
  uint16_t cap = 0;
  AdaptState adapt{};
  uint64_t pmc[kNumPmc] = {0, 0, 0, 0};  // last per-tenant deltas (sdom->pmc)
  uint64_t spinlock_latency = 0, spinlock_metric_update = 0, spinlock_count = 0, report_total = 0;
  uint64_t lock_hold_ns = 0, lock_hold_count = 0;
  uint64_t pending_requests = 0;
  uint64_t cache_miss_rate = 0, cpi = 0;
  uint64_t rate_ewma = 0;  // smoothed miss rate (alpha 1/4) for contention classes
  uint64_t bound_periods = 0, bound_min = 0, bound_max = 0;  // measured periods / at min_us / at max_us
  // The quantum the dispatcher actually gave the tenant (s_timer, before the
  // quantum_align grid and measurement tenures): last one, and since when
  // (the reported quantum is the dispatched one; the
  // adaptive target stays in adapt.tslice_us)
  uint32_t q_disp_us = 0;
  // region virtual time (boot region_vt): partition-ns the tenant ran in its
  // time-shared class region, x 256 / weight
  int64_t rvt = 0;
  AtcState atc{};
};

struct CPcpu : SchedPartData {
  std::list<int> runq;
  uint32_t runq_sort_last = 0;
  int ticker = -1;
  int metric_ticker = -1;
  uint32_t tick = 0;
  int idle_bias = 0;  int64_t rvt_mark = 0;  // region virtual time: the current runner is accounted up to here
};

class CreditScheduler : public Scheduler {
 public:
  CreditScheduler(Engine& e, int pool, Mode m) : Scheduler(e, pool), mode_(m) {}

  const char* name() const override {
    return mode_ == Mode::ATC ? "SMP Credit Scheduler (ATC)"
                              : (mode_ == Mode::PBS ? "SMP Credit Scheduler (PBS)" : "SMP Credit Scheduler");
  }
  const char* opt_name() const override {
    return mode_ == Mode::ATC ? "atc" : (mode_ == Mode::PBS ? "credit" : (mode_ == Mode::CLASSQ ? "credit-classq" : "credit-fixed"));
  }

  // ------------------------------------------------------------- init ----
  int init() override {
    int ts = E.boot.tslice_us;
    if (mode_ == Mode::ATC) ts = (int)E.atc_params.default_us;
    if (ts > GPBS_TSLICE_UMAX || ts < GPBS_TSLICE_UMIN) {
      E.printk(fmt("WARNING: sched_credit_tslice_us outside of valid range [%d,%d].\n Resetting to default %u\n",
                   GPBS_TSLICE_UMIN, GPBS_TSLICE_UMAX, 100));
      ts = 100;
    }
    int rl = E.boot.ratelimit_us;
    if (rl > GPBS_RATELIMIT_MAX || (rl < GPBS_RATELIMIT_MIN && rl != 0)) {
      E.printk(fmt("WARNING: sched_ratelimit_us outside of valid range [%d,%d].\n Resetting to default %u\n",
                   GPBS_RATELIMIT_MIN, GPBS_RATELIMIT_MAX, 1000));
      rl = 1000;
    }
    tslice_us_ = (uint32_t)ts;
    recompute();
    if (rl > ts) {
      E.printk("WARNING: sched_ratelimit_us >sched_credit_tslice_us is undefined\nSetting ratelimit_us to tslice\n");
      ratelimit_us_ = tslice_us_;
    } else {
      ratelimit_us_ = (uint32_t)rl;
    }
    master_ticker_ = E.timer_init([this](int64_t n) { acct(n); });
    slice_ticker_ = E.timer_init([this](int64_t n) { dynamic_time_slice(n); });
    return 0;
  }

  void deinit() override {
    E.timer_kill(master_ticker_);
    E.timer_kill(slice_ticker_);
    master_ticker_ = slice_ticker_ = -1;
  }

  void recompute() {
    ticks_per_tslice_ = 3;
    if (E.adapt_params.ticks_per_tslice) ticks_per_tslice_ = E.adapt_params.ticks_per_tslice;
    if (tslice_us_ < ticks_per_tslice_) ticks_per_tslice_ = 1;
    tick_period_us_ = tslice_us_ / ticks_per_tslice_;
    credits_per_tslice_ = tslice_us_;  // CSCHED_CREDIT_PER_US * tslice
    credit_ = ncpus_ * credits_per_tslice_;
  }

  CPcpu& pc(int cpu) { return *static_cast<CPcpu*>(E.parts[cpu]->priv.get()); }
  CSlot& sv(Slot& v) { return *static_cast<CSlot*>(v.priv.get()); }
  CSlot& sv(int id) { return sv(*E.slots[id]); }
  CDom& sd(Tenant& d) { return *static_cast<CDom*>(d.priv.get()); }
  CDom& sd_of(Slot& v) { return sd(*E.tenants[v.tenant]); }

  // ------------------------------------------------------- the quantum --
  // A time-shared class region (class_budget 1, budget_shared): every tenant
  // laid out there holds every partition of it, and they take turns.
  static int region_cls(const Tenant& t) { return t.lay_cls >= 0 ? t.lay_cls : t.cls; }
  static bool shared_region(const Tenant& t) { return t.budget_shared && region_cls(t) >= 0; }
  bool cosharer(const Tenant& t, const Tenant& o) const {
    return o.alive && o.priv && o.pool == t.pool && shared_region(o) && region_cls(o) == region_cls(t) &&
           o.budget_ctx != 0;
  }
  // credit-classq: the class's bound (unknown class: the global quantum)
  uint32_t classq_us(const Tenant& t) const {
    return t.cls == 1 ? E.adapt_params.max_us : (t.cls == 0 ? E.adapt_params.min_us : tslice_us_);
  }
  // The policy's own quantum for a tenant: PBS its adaptive tslice (:1796-1804),
  // classq its class's bound, otherwise the pool's global quantum.
  uint32_t target_us(Tenant& t) {
    if (mode_ == Mode::PBS) return sd(t).adapt.tslice_us;
    if (mode_ == Mode::CLASSQ) return classq_us(t);
    return tslice_us_;
  }
  // Per-tenant switch-cost floor (boot switch_floor_x): a tenant whose every
  // switch costs c (its revoked tiles drain, then its grid ramps back in --
  // measured by the GPU runtime per tenant) loses c / q of each turn, so its
  // quantum is kept at >= x * c (x = 25: at most 4 % of a turn lost).  The
  // GPU's stand-in for the reference's cache-warmth argument (a cache-
  // sensitive domain gets the longer slice, :294-300): what a switch costs is
  // measured per tenant instead of inferred from its miss rate.
  uint32_t switch_floor_us(const Tenant& t) const {
    if (E.boot.switch_floor_x <= 0 || !t.sw_cost_us) return 0;
    const uint32_t cap = E.boot.switch_floor_max_us > 0 ? (uint32_t)E.boot.switch_floor_max_us : E.adapt_params.max_us;
    uint64_t f = std::min<uint64_t>((uint64_t)t.sw_cost_us * (uint64_t)E.boot.switch_floor_x, cap);
    if (E.boot.quantum_align_us > 0) {
      const uint64_t a = (uint64_t)E.boot.quantum_align_us;
      f = (f + a - 1) / a * a;
    }
    return (uint32_t)f;
  }
  // SLO cap (boot slo_cap): a co-sharer of a region that holds a tenant with a
  // latency target gets at most that target minus one ratelimit as its
  // quantum, so a request of the target tenant that arrives during the
  // co-sharer's turn (and cannot preempt it: no BOOST for an OVER slot, or a
  // strict_ref ratelimit hold) waits at most the target for the region.
  uint32_t slo_cap_us(const Tenant& t) {
    uint32_t cap = UINT32_MAX;
    for (auto& tp : E.tenants)
      if (tp && tp.get() != &t && tp->slo_us && cosharer(t, *tp))
        cap = std::min<uint32_t>(cap, tp->slo_us > ratelimit_us_ ? tp->slo_us - ratelimit_us_ : tp->slo_us);
    return cap;
  }
  // The quantum a slot of tenant t is dispatched with (the s_timer of
  // :1796-1804).  Outside a time-shared region: the policy's own quantum.
  // Inside one, per tenant (boot region_q 0):
  //   PBS     its adaptive quantum, at least its switch-cost floor;
  //   classq  its class's bound, at least shared_q_us (the classq+floor
  //           ablation) when that is set;
  //   others  the global quantum;
  // then capped by a latency-target co-sharer (slo_cap), never below min_us.
  // region_q 1 keeps round 5's region quantum: the largest adaptive quantum
  // among the co-sharers, floored at shared_q_us -- every co-sharer the same.
  // Per-tenant quanta stay weight-fair through the region's virtual time
  // (region_pick): a tenant with twice the quantum gets half the turns.
  uint32_t quantum_us(Tenant& t) {
    uint32_t q = target_us(t);
    if (!shared_region(t)) return q;
    if (mode_ == Mode::PBS && E.boot.region_q) {
      for (auto& tp : E.tenants)
        if (tp && tp->priv && cosharer(t, *tp)) q = std::max(q, sd(*tp).adapt.tslice_us);
      if (E.boot.shared_q_us > 0) q = std::max(q, (uint32_t)E.boot.shared_q_us);
      return q;
    }
    if (mode_ == Mode::PBS) q = std::max(q, switch_floor_us(t));
    if (mode_ == Mode::CLASSQ && E.boot.shared_q_us > 0) q = std::max(q, (uint32_t)E.boot.shared_q_us);
    if (E.boot.slo_cap) q = std::max(std::min(q, slo_cap_us(t)), std::min(q, E.adapt_params.min_us));
    return q;
  }
  // What tenant_info / bound stats report: the quantum the tenant is
  // dispatched with now (the s_timer quantum; the last one actually given is
  // CDom::q_disp_us, tenant_info.last_dispatch_us).
  uint32_t reported_us(Tenant& t) { return quantum_us(t); }
  Slot& curr(int cpu) { return E.curr_of(cpu); }
  Mask online() { return E.pools[pool_]->cpus; }
  // Another runnable slot of v's tenant on `cpu` (running there or queued).
  bool sibling_on(int cpu, const Slot& v) {
    const Slot& c = curr(cpu);
    if (&c != &v && !c.is_idle() && c.tenant == v.tenant && E.runnable(c)) return true;
    for (int sid : pc(cpu).runq) {
      const Slot& w = *E.slots[sid];
      if (&w != &v && w.tenant == v.tenant) return true;
    }
    return false;
  }

  void alloc_pdata(int cpu) override {
    auto p = std::make_unique<CPcpu>();
    credit_ += credits_per_tslice_;
    ncpus_++;
    cpus_.set(cpu);
    const int64_t n = E.now();
    if (ncpus_ == 1) {
      master_ = cpu;
      E.timer_set(master_ticker_, n + (int64_t)tslice_us_ * 1000);
      E.timer_set(slice_ticker_, n + (int64_t)slice_period_us() * 1000);
    }
    p->ticker = E.timer_init([this, cpu](int64_t t) { tick(cpu, t); });
    p->metric_ticker = E.timer_init([this, cpu](int64_t t) { metric_tick(cpu, t); });
    E.timer_set(p->ticker, n + std::max<int64_t>(1, tick_period_us_) * 1000);
    E.timer_set(p->metric_ticker, n + (int64_t)E.boot.metric_period_us * 1000);
    p->runq_sort_last = runq_sort_;
    p->idle_bias = kMaxPartitions - 1;
    E.parts[cpu]->priv = std::move(p);
    idlers_.set(cpu);
  }

  void free_pdata(int cpu) override {
    CPcpu& p = pc(cpu);
    credit_ -= credits_per_tslice_;
    ncpus_--;
    idlers_.clear(cpu);
    cpus_.clear(cpu);
    if (master_ == cpu && ncpus_ > 0) master_ = cpus_.first();  // migrate_timer(master/slice)
    E.timer_kill(p.ticker);
    E.timer_kill(p.metric_ticker);
    if (ncpus_ == 0) {
      E.timer_stop(master_ticker_);
      E.timer_stop(slice_ticker_);
    }
    for (int sid : p.runq) sv(sid).runq_cpu = -1;
    E.parts[cpu]->priv.reset();
  }

  int init_domain(Tenant& d) override {
    auto s = std::make_unique<CDom>();
    // The reference starts every domain at 100 us (csched_dom_init :1217),
    // its profile's floor.  Q15: under a profile whose floor is higher (MI355X:
    // 1 ms) that start value sat below the floor, and a tenant whose miss rate
    // never settled into the stable band kept it -- neither the window nor the
    // unstable branch decrements a memory-bound tenant, and only dec() clamps
    // -- so a time-shared HBM tenant ran 100 us quanta that were all switch
    // and drain (0.05 of solo next to a reduce-copy tenant at 11 ms quanta).
    // Start at the floor when it is above 100 us.
    const uint32_t q0 = std::max<uint32_t>(100, E.adapt_params.min_us);
    adapt_init(s->adapt, E.adapt_params, mode_ == Mode::FIXED ? tslice_us_ : q0);
    atc_init(s->atc, E.atc_params);
    d.priv = std::move(s);
    return 0;
  }
  void destroy_domain(Tenant& d) override { d.priv.reset(); }

  void alloc_vdata(Slot& v) override {
    auto s = std::make_unique<CSlot>();
    s->pri = v.is_idle() ? PRI_IDLE : PRI_UNDER;
    v.priv = std::move(s);
    // (class_budget layouts place every slot themselves: one per partition
    // of the tenant's SE budget.  ATC's hard-affinity spreading on top pinned
    // slots away from their class homes -- 4mix under atc measured 0.58 with
    // half the partitions idle, s29.)
    if (mode_ == Mode::ATC && !v.is_idle() && !(E.boot.class_budget && E.boot.class_split > 1)) atc_place(v);
  }

  // ATC placement (X:xen/common/sched_credit_atc.c:634-651, called from
  // alloc_vdata :1171): a new slot goes to the least-loaded partition (runq
  // length, :572-632) not already used by a sibling slot, and every slot of
  // the tenant is then hard-pinned away from its siblings' partitions
  // (set_vcpu_affinity :545-570), so a tenant's slots never queue behind one
  // another -- the ATC answer to lock-holder preemption.
  void atc_place(Slot& v) {
    Tenant* t = E.tenant(v.tenant);
    if (!t || cpus_.empty()) return;
    Mask used;
    for (int sid : t->slots)
      if (sid != v.id && E.slots[sid]) used.set(E.slots[sid]->processor);
    Mask cand = (cpus_ & v.affinity).andnot(used);
    if (cand.empty()) cand = cpus_ & v.affinity;
    if (cand.empty()) cand = cpus_;
    int best = cand.first();
    size_t best_load = pc(best).runq.size();
    for (int c = cand.first(); c >= 0; c = cand.next(c + 1))
      if (pc(c).runq.size() < best_load) {
        best = c;
        best_load = pc(c).runq.size();
      }
    v.processor = best;
    used.set(best);
    for (int sid : t->slots) {
      if (!E.slots[sid]) continue;
      Slot& w = *E.slots[sid];
      Mask aff = cpus_.andnot(used);
      aff.set(w.processor);
      w.affinity = aff;
    }
  }

  void insert_vcpu(Slot& v) override {
    CSlot& s = sv(v);
    if (s.runq_cpu < 0 && E.runnable(v) && !v.is_running) runq_insert(v.processor, v);
  }

  void remove_vcpu(Slot& v) override {
    CSlot& s = sv(v);
    if (s.runq_cpu >= 0) runq_remove(v);
    if (s.active) acct_stop_locked(v);
  }

  // ------------------------------------------------------------ runq ----
  void runq_insert(int cpu, Slot& v) {
    CSlot& s = sv(v);
    auto& rq = pc(cpu).runq;
    auto it = rq.begin();
    for (; it != rq.end(); ++it)
      if (s.pri > sv(*it).pri) break;
    // A yielding slot goes behind one lower-priority runnable slot.
    if ((s.flags & FLAG_YIELD) && it != rq.end() && sv(*it).pri > PRI_IDLE) ++it;
    rq.insert(it, v.id);
    s.runq_cpu = cpu;
  }

  void runq_remove(Slot& v) {
    CSlot& s = sv(v);
    pc(s.runq_cpu).runq.remove(v.id);
    s.runq_cpu = -1;
  }

  void burn_credits(Slot& v, int64_t now) {
    CSlot& s = sv(v);
    int64_t delta = now - s.start_time;
    if (delta <= 0) return;
    // credits = round(delta[ns] * 1000/ms) -> 1 credit per us
    uint32_t credits = (uint32_t)((delta * 1000 + 500000) / 1000000);
    s.credit -= (int32_t)credits;
    s.start_time += (int64_t)credits * 1000000 / 1000;
  }

  void tickle(int cpu, Slot& nw) {
    Slot& cur = curr(cpu);
    CSlot& cs = sv(cur);
    CSlot& ns = sv(nw);
    Mask mask;
    if (ns.pri > cs.pri) {
      if (cs.pri == PRI_IDLE)
        E.perfc.incr(PC_tickle_local_idler);
      else if (cs.pri == PRI_OVER)
        E.perfc.incr(PC_tickle_local_over);
      else if (cs.pri == PRI_UNDER)
        E.perfc.incr(PC_tickle_local_under);
      else
        E.perfc.incr(PC_tickle_local_other);
      mask.set(cpu);
    }
    if (cs.pri > PRI_IDLE) {
      if (idlers_.empty()) {
        E.perfc.incr(PC_tickle_idlers_none);
      } else {
        Mask idle_mask = idlers_ & nw.affinity & online();
        if (!idle_mask.empty()) {
          E.perfc.incr(PC_tickle_idlers_some);
          if (E.boot.tickle_one_idle) {
            last_tickle_cpu_ = idle_mask.cycle(last_tickle_cpu_);
            mask.set(last_tickle_cpu_);
          } else {
            mask = mask | idle_mask;
          }
        }
        mask = mask & nw.affinity;
      }
    }
    for (int c = mask.first(); c >= 0; c = mask.next(c + 1)) E.raise_softirq(c);
  }

  // --------------------------------------------------------- cpu pick ----
  Mask sibling_mask(int cpu) {  // partitions sharing an XCD (SMT-sibling analog)
    Mask m;
    const Partition& P = *E.parts[cpu];
    for (int c = cpus_.first(); c >= 0; c = cpus_.next(c + 1))
      if (E.parts[c]->gpu == P.gpu && E.parts[c]->xcd == P.xcd) m.set(c);
    m.set(cpu);
    return m;
  }
  Mask core_mask(int cpu) {  // partitions on the same GPU (socket analog)
    Mask m;
    const Partition& P = *E.parts[cpu];
    for (int c = cpus_.first(); c >= 0; c = cpus_.next(c + 1))
      if (E.parts[c]->gpu == P.gpu) m.set(c);
    m.set(cpu);
    return m;
  }

  int cpu_pick(Slot& v, bool commit) {
    Mask cpus = online() & v.affinity;
    if (cpus.empty()) cpus = online();
    if (cpus.empty()) return v.processor;
    // Soft affinity (contention class): restrict to it when it is usable --
    // it contains the current partition or an idler (Xen 4.5's soft step).
    if (!v.soft.empty()) {
      Mask sc = cpus & v.soft;
      if (!sc.empty() && (sc.test(v.processor) || !(sc & idlers_).empty())) cpus = sc;
    }
    int cpu = cpus.test(v.processor) ? v.processor : cpus.cycle(v.processor);
    Mask idlers = idlers_;
    idlers.set(cpu);
    cpus = cpus & idlers;
    cpus.clear(cpu);
    CPcpu* spc = nullptr;
    while (!cpus.empty()) {
      int nxt = cpus.cycle(cpu);
      Mask cpu_idlers, nxt_idlers;
      int factor;
      if (E.parts[cpu]->gpu == E.parts[nxt]->gpu) {
        factor = 1;
        cpu_idlers = idlers & sibling_mask(cpu);
        nxt_idlers = idlers & sibling_mask(nxt);
      } else {
        factor = 2;  // migrate across GPUs only if twice as idle
        cpu_idlers = idlers & core_mask(cpu);
        nxt_idlers = idlers & core_mask(nxt);
      }
      int wc = cpu_idlers.weight(), wn = nxt_idlers.weight();
      if (E.boot.smt_power_savings ? wc > wn : wc * factor < wn) {
        nxt_idlers = cpus & nxt_idlers;
        spc = &pc(nxt);
        cpu = nxt_idlers.cycle(spc->idle_bias);
        cpus = cpus.andnot(sibling_mask(cpu));
      } else {
        cpus = cpus.andnot(nxt_idlers);
      }
    }
    if (commit && spc) spc->idle_bias = cpu;
    return cpu;
  }
  int pick_cpu(Slot& v) override { return cpu_pick(v, true); }

  // ------------------------------------------------------- accounting ----
  void acct_start(Slot& v) {
    CSlot& s = sv(v);
    CDom& d = sd_of(v);
    if (!s.active) {
      s.stats.state_active++;
      E.perfc.incr(PC_acct_vcpu_active);
      d.active_vcpu_count++;
      d.active_vcpu.push_front(v.id);
      s.active = true;
      weight_ += d.weight;
      if (!d.on_active) {
        active_sdom_.push_front(v.tenant);
        d.on_active = true;
      }
    }
  }

  void acct_stop_locked(Slot& v) {
    CSlot& s = sv(v);
    CDom& d = sd_of(v);
    s.stats.state_idle++;
    E.perfc.incr(PC_acct_vcpu_idle);
    d.active_vcpu_count--;
    d.active_vcpu.remove(v.id);
    s.active = false;
    weight_ -= d.weight;
    if (d.active_vcpu.empty()) {
      active_sdom_.remove(v.tenant);
      d.on_active = false;
    }
  }

  void vcpu_acct(int cpu, int64_t now) {
    Slot& v = curr(cpu);
    CSlot& s = sv(v);
    if (s.pri == PRI_BOOST) s.pri = PRI_UNDER;
    if (!v.is_idle()) burn_credits(v, now);
    if (!s.active) {
      acct_start(v);
    } else if (cpu_pick(v, false) != cpu) {
      s.stats.migrate_r++;
      E.perfc.incr(PC_migrate_running);
      v.pause_flags |= VPF_MIGRATING;
      E.raise_softirq(cpu);
    }
  }

  void acct(int64_t now) {
    uint64_t weight_total = weight_;
    uint64_t credit_total = credit_;
    if (credit_balance_ < 0) {
      credit_total += (uint64_t)(-credit_balance_);
      E.perfc.incr(PC_acct_balance);
    }
    if (weight_total == 0) {
      credit_balance_ = 0;
      E.perfc.incr(PC_acct_no_work);
      E.timer_set(master_ticker_, now + (int64_t)tslice_us_ * 1000);
      return;
    }
    E.perfc.incr(PC_acct_run);
    uint64_t weight_left = weight_total;
    int64_t credit_balance = 0;
    bool credit_xtra = false;
    uint64_t credit_cap = 0;
    const uint64_t cpt = credits_per_tslice_;

    std::vector<int> doms(active_sdom_.begin(), active_sdom_.end());
    for (int tid : doms) {
      Tenant& dom = *E.tenants[tid];
      CDom& d = sd(dom);
      if (!d.on_active) continue;
      const uint64_t n = d.active_vcpu_count;
      const uint64_t w = d.weight;
      weight_left -= w * n;
      uint64_t credit_peak = n * cpt;
      if (credit_balance_ < 0) credit_peak += ((uint64_t)(-credit_balance_) * w * n + (weight_total - 1)) / weight_total;
      if (d.cap != 0) {
        credit_cap = ((uint64_t)d.cap * cpt + 99) / 100;
        if (credit_cap < credit_peak) credit_peak = credit_cap;
        credit_cap = (credit_cap + (n - 1)) / n;
      }
      uint64_t credit_fair = (credit_total * w * n + (weight_total - 1)) / weight_total;
      if (credit_fair < credit_peak) {
        credit_xtra = true;
      } else {
        if (weight_left != 0)  // give other domains a chance at unused credits
          credit_total += ((credit_fair - credit_peak) * weight_total + (weight_left - 1)) / weight_left;
        if (credit_xtra) {
          E.perfc.incr(PC_acct_reorder);
          active_sdom_.remove(tid);
          active_sdom_.push_front(tid);
        }
        credit_fair = credit_peak;
      }
      credit_fair = (credit_fair + (n - 1)) / n;  // per slot

      std::vector<int> vs(d.active_vcpu.begin(), d.active_vcpu.end());
      for (int sid : vs) {
        Slot& v = *E.slots[sid];
        CSlot& s = sv(v);
        s.credit += (int32_t)credit_fair;
        int32_t credit = s.credit;
        // A BOOSTed waker that has not been dispatched yet keeps BOOST (gpbs
        // extension; Xen's acct walks only vCPUs that ran since their last
        // activation, here a latency tenant's slots stay on the active list
        // between requests): demoting it here put a woken in-region latency
        // tenant behind its co-sharers' gang rotation -- a request arriving
        // during a ratelimit hold waited 16-20 ms on MI355X (slo mix traces,
        // profiles/r6/slo_diag_summary.txt).  Its first tick while running
        // demotes it (vcpu_acct), as before.
        const bool waker = s.pri == PRI_BOOST && !v.is_running && !E.adapt_params.strict_ref;
        if (credit < 0) {
          s.pri = waker ? PRI_BOOST : PRI_OVER;
          // Park running slots of capped-out tenants (launch gate closes).
          if (d.cap != 0 && credit < -(int32_t)credit_cap && !(s.flags & FLAG_PARKED)) {
            E.perfc.incr(PC_vcpu_park);
            E.vcpu_pause(v);
            s.flags |= FLAG_PARKED;
            E.emit(TRC_PARK, v.processor, v.tenant, v.index, 1);
            if (E.actuator_ops.on_park) E.actuator_ops.on_park(E.actuator_ops.user, v.tenant, v.index, 1);
          }
          if (credit < -(int32_t)cpt) {  // lower bound
            E.perfc.incr(PC_acct_min_credit);
            credit = -(int32_t)cpt;
            s.credit = credit;
          }
        } else {
          s.pri = waker ? PRI_BOOST : PRI_UNDER;
          if (s.flags & FLAG_PARKED) {
            E.perfc.incr(PC_vcpu_unpark);
            E.vcpu_unpause(v);
            s.flags &= ~FLAG_PARKED;
            E.emit(TRC_PARK, v.processor, v.tenant, v.index, 0);
            if (E.actuator_ops.on_park) E.actuator_ops.on_park(E.actuator_ops.user, v.tenant, v.index, 0);
          }
          if (E.boot.dom0_quirk) {
            // P1g (:1486-1500): ceiling compared at /100 granularity; tenant 0
            // (the control tenant) leaves the active list only with >=2 active
            // slots and keeps its credit; others halve and stay active.
            if (credit / 100 > (int32_t)cpt / 100 && tid == 0) {
              if (d.active_vcpu_count >= 2) acct_stop_locked(v);
              s.credit = credit;
            } else if (credit / 100 > (int32_t)cpt / 100 && tid != 0) {
              credit /= 2;
              s.credit = credit;
            }
          } else if (credit > (int32_t)cpt) {  // upstream: stop earning, halve
            acct_stop_locked(v);
            credit /= 2;
            s.credit = credit;
          }
        }
        s.stats.credit_last = credit;
        s.stats.credit_incr = (uint32_t)credit_fair;
        credit_balance += credit;
      }
    }
    credit_balance_ = (int32_t)credit_balance;
    runq_sort_++;
    E.emit(TRC_ACCT, master_, (uint32_t)pool_, (uint32_t)weight_total, (uint32_t)credit_total,
           (uint32_t)credit_balance_);
    E.timer_set(master_ticker_, now + (int64_t)tslice_us_ * 1000);
  }

  void runq_sort(int cpu) {
    CPcpu& p = pc(cpu);
    if (p.runq_sort_last == runq_sort_) return;
    p.runq_sort_last = runq_sort_;
    std::stable_partition(p.runq.begin(), p.runq.end(), [this](int sid) { return sv(sid).pri >= PRI_UNDER; });
  }

  void tick(int cpu, int64_t now) {
    CPcpu& p = pc(cpu);
    p.tick++;
    Slot& c = curr(cpu);
    if (!c.is_idle()) vcpu_acct(cpu, now);
    if ((int)tslice_us_ > E.boot.pmu_refresh_us) E.pmu_refresh(curr(cpu));
    runq_sort(cpu);
    Slot& c2 = curr(cpu);
    uint32_t period = tick_period_us_;
    if (!c2.is_idle() && mode_ == Mode::PBS) period = sd_of(c2).adapt.tick_period_us;
    if (!c2.is_idle() && mode_ == Mode::CLASSQ)
      period = classq_us(*E.tenants[c2.tenant]) / std::max<uint32_t>(1, E.adapt_params.ticks_per_tslice);
    E.timer_set(p.ticker, now + (int64_t)std::max<uint32_t>(1, period) * 1000);
  }

  // ---------------------------------------------------- PBS metric loop --
  void metric_tick(int cpu, int64_t now) {
    CPcpu& p = pc(cpu);
    if ((int)tslice_us_ <= E.boot.pmu_refresh_us) E.pmu_refresh(curr(cpu));
    if (cpu == master_) dom_metric_update(now);
    E.timer_set(p.metric_ticker, now + (int64_t)E.boot.metric_period_us * 1000);
  }

  void dom_metric_update(int64_t now) {
    E.perfc.incr(PC_metric_tick);
    std::vector<int> ids;
    for (auto& t : E.tenants)
      if (t && t->alive && t->pool == pool_ && t->priv) ids.push_back(t->id);
    if (ids.empty()) return;
    const size_t n = ids.size();
    std::vector<uint64_t> deltas(4 * n, 0), ssum(n), scnt(n);
    bool have = false;
    if (E.counter_ops.tenant_deltas) {
      have = E.counter_ops.tenant_deltas(E.counter_ops.user, (int)n, ids.data(), deltas.data()) == 0;
      if (!have) E.perfc.incr(PC_counter_stale);
    }
    for (size_t k = 0; k < n; ++k) {
      Tenant& dom = *E.tenants[ids[k]];
      CDom& d = sd(dom);
      d.pending_requests = dom.pending_requests;  // P7
      dom.pending_requests = 0;
      // The per-slot snapshots advance on every tick whichever source supplied
      // the deltas, so a later host fallback never reports one delta spanning
      // all the periods the device backend covered.
      {
        for (int sid : dom.slots) {
          Slot& v = *E.slots[sid];
          CSlot& s = sv(v);
          for (int i = 0; i < kNumPmc; ++i) {
            if (v.pmc[i] < s.prev_pmc[i]) {  // Q5: counter reset -> skip sample
              if (!have) E.perfc.incr(PC_counter_reset);
            } else if (!have) {
              deltas[4 * k + i] += v.pmc[i] - s.prev_pmc[i];
            }
            s.prev_pmc[i] = v.pmc[i];
          }
        }
      }
      for (int i = 0; i < kNumPmc; ++i) {
        d.pmc[i] = deltas[4 * k + i];
        dom.vpmu_total[i] += deltas[4 * k + i];
      }
      ssum[k] = d.spinlock_metric_update;
      scnt[k] = d.spinlock_count;
    }
    if (mode_ == Mode::PBS && E.counter_ops.adapt_launch && E.counter_ops.adapt_harvest) {
      adapt_async(ids, deltas, ssum, scnt);
    } else if (mode_ == Mode::PBS) {
      std::vector<AdaptState> before(n);
      for (size_t k = 0; k < n; ++k) before[k] = sd(*E.tenants[ids[k]]).adapt;
      bool dev = false;
      if (E.counter_ops.adapt_batch) {
        std::vector<gpbs_adapt_state_t> st(n);
        for (size_t k = 0; k < n; ++k) std::memcpy(&st[k], &before[k], sizeof(AdaptState));
        dev = E.counter_ops.adapt_batch(E.counter_ops.user, (int)n, ids.data(), deltas.data(), ssum.data(), scnt.data(),
                                        st.data(), reinterpret_cast<const gpbs_adapt_params_t*>(&E.adapt_params)) == 0;
        if (dev)
          for (size_t k = 0; k < n; ++k) std::memcpy(&sd(*E.tenants[ids[k]]).adapt, &st[k], sizeof(AdaptState));
      }
      for (size_t k = 0; k < n; ++k) {
        CDom& d = sd(*E.tenants[ids[k]]);
        bool rearm = false;
        int dir;
        // Q14 idle-sample rule (gpbs extension): a tenant that retired no
        // instructions this period was not dispatched (it idles between
        // work quotas, or its counters have not been harvested yet).  The
        // reference feeds curr = 0 here, which the detector reads as
        // "not cache-bound" and answers with DEC/re-arm, driving a
        // memory-bound tenant that merely paused to the minimum quantum.
        // The sample is skipped instead, as Q5 skips counter resets.
        if (E.boot.idle_skip && deltas[4 * k + 0] == 0) {
          if (dev) d.adapt = before[k];
          E.perfc.incr(PC_adapt_idle_skip);
          continue;
        }
        if (!dev) {
          dir = adapt_update(d.adapt, E.adapt_params, deltas[4 * k + 0], deltas[4 * k + 3], ssum[k], scnt[k], &rearm);
        } else {
          dir = d.adapt.tslice_us > before[k].tslice_us ? 1 : (d.adapt.tslice_us < before[k].tslice_us ? -1 : 0);
          rearm = d.adapt.window_left == kWindow - 1 && before[k].window_left == 0;
        }
        adapt_account(ids[k], before[k], d.adapt, dir, rearm);
      }
    }
    for (size_t k = 0; k < n; ++k) {
      CDom& d = sd(*E.tenants[ids[k]]);
      const uint64_t inst = d.pmc[0], cyc = d.pmc[1], miss = d.pmc[3];
      // Q14 (idle_skip): a period without instructions -- no dispatch, or no
      // exclusive-ownership counter window -- keeps the last measured rates
      // instead of reporting 0 for the tenant
      if (inst || !E.boot.idle_skip) {
        d.cache_miss_rate = inst ? miss * 100000 / inst : 0;  // Q3 fix: per tenant
        d.cpi = inst ? cyc * 1000 / inst : 0;
      }
      if (inst)  // class_fall: follow a drop at alpha 1/2 (rises cross the threshold in one sample anyway)
        d.rate_ewma = (E.boot.class_fall && d.cache_miss_rate < d.rate_ewma)
                          ? (d.rate_ewma + d.cache_miss_rate) / 2
                          : (3 * d.rate_ewma + d.cache_miss_rate) / 4;
      E.emit(TRC_METRIC, master_, (uint32_t)ids[k], (uint32_t)inst, (uint32_t)miss, (uint32_t)d.cache_miss_rate);
      if (inst) {  // a measured period: where the quantum sits
        const uint32_t q = reported_us(*E.tenants[ids[k]]);  // the dispatched quantum
        d.bound_periods++;
        d.bound_min += q <= E.adapt_params.min_us;
        d.bound_max += q >= E.adapt_params.max_us;
      }
      d.spinlock_metric_update = 0;
      d.spinlock_count = 0;
    }
  }

  void adapt_account(int id, const AdaptState& before, const AdaptState& after, int dir, bool rearm) {
    if (dir > 0) E.perfc.incr(PC_adapt_inc);
    if (dir < 0) E.perfc.incr(PC_adapt_dec);
    if (rearm) E.perfc.incr(PC_adapt_rearm);
    if (dir || rearm)
      E.emit(TRC_ADAPT, master_, (uint32_t)id, before.tslice_us, after.tslice_us,
             (after.phase << 24) | ((uint32_t)after.last_err & 0xffffff));
  }

  // Asynchronous device adaptation: period k's PBS update runs on the GPU
  // (k_adapt) while the dispatcher goes on; tick k+1 applies it, then starts
  // k+1's.  Each launch starts from the states the previous one produced, so
  // the sequence of states is exactly the host's, one metric period late.  A
  // launch still running at the next tick (a tail: the GPU was full) is
  // recomputed on the host from its saved inputs and its result discarded.
  struct AsyncIn {
    int id;
    AdaptState before;
    uint64_t inst, miss, ssum, scnt;
  };
  std::vector<AsyncIn> async_in_;
  bool async_pending_ = false;

  void async_apply(int id, const AdaptState& before, const AdaptState& after) {
    Tenant* t = E.tenant(id);
    if (!t || !t->alive || !t->priv || t->pool != pool_) return;
    // the state moved since the launch (a class-change seed, an API set):
    // the newer state wins over a result computed from the old one
    if (std::memcmp(&sd(*t).adapt, &before, sizeof(before)) != 0) return;
    sd(*t).adapt = after;
    const int dir = after.tslice_us > before.tslice_us ? 1 : (after.tslice_us < before.tslice_us ? -1 : 0);
    const bool rearm = after.window_left == kWindow - 1 && before.window_left == 0;
    adapt_account(id, before, after, dir, rearm);
  }

  void adapt_async(const std::vector<int>& ids, const std::vector<uint64_t>& deltas, const std::vector<uint64_t>& ssum,
                   const std::vector<uint64_t>& scnt) {
    const gpbs_adapt_params_t* pp = reinterpret_cast<const gpbs_adapt_params_t*>(&E.adapt_params);
    // 1. the previous period's results
    if (async_pending_) {
      std::vector<int> hid(async_in_.size() + 1);
      std::vector<gpbs_adapt_state_t> hst(async_in_.size() + 1);
      for (size_t i = 0; i < async_in_.size(); ++i) hid[i] = async_in_[i].id;  // in: this pool's launch
      int nh = E.counter_ops.adapt_harvest(E.counter_ops.user, (int)async_in_.size(), hid.data(), hst.data());
      // a result for other tenants (another pool's launch) is never applied
      for (int i = 0; i < nh && nh >= 0; ++i)
        if (i >= (int)async_in_.size() || hid[i] != async_in_[i].id) nh = -22;
      if (nh == (int)async_in_.size()) {
        for (int i = 0; i < nh && i < (int)async_in_.size(); ++i) {
          AdaptState after;
          std::memcpy(&after, &hst[i], sizeof(after));
          async_apply(async_in_[i].id, async_in_[i].before, after);
        }
      } else {  // late: the host recomputes that period (bit-identical), the device result is dropped
        E.perfc.incr(PC_adapt_late);
        for (auto& a : async_in_) {
          AdaptState st = a.before;
          bool rearm = false;
          adapt_update(st, E.adapt_params, a.inst, a.miss, a.ssum, a.scnt, &rearm);
          async_apply(a.id, a.before, st);
        }
      }
      async_pending_ = false;
    }
    // 2. this period: every non-idle tenant (Q14), from its current state
    async_in_.clear();
    std::vector<int> lid;
    std::vector<uint64_t> ld, ls, lc;
    std::vector<gpbs_adapt_state_t> lst;
    for (size_t k = 0; k < ids.size(); ++k) {
      if (E.boot.idle_skip && deltas[4 * k + 0] == 0) {
        E.perfc.incr(PC_adapt_idle_skip);
        continue;
      }
      CDom& d = sd(*E.tenants[ids[k]]);
      async_in_.push_back({ids[k], d.adapt, deltas[4 * k + 0], deltas[4 * k + 3], ssum[k], scnt[k]});
      lid.push_back(ids[k]);
      for (int i = 0; i < 4; ++i) ld.push_back(deltas[4 * k + i]);
      ls.push_back(ssum[k]);
      lc.push_back(scnt[k]);
      gpbs_adapt_state_t g;
      std::memcpy(&g, &d.adapt, sizeof(g));
      lst.push_back(g);
    }
    if (async_in_.empty()) return;
    if (E.counter_ops.adapt_launch(E.counter_ops.user, (int)lid.size(), lid.data(), ld.data(), ls.data(), lc.data(),
                                   lst.data(), pp) == 0) {
      async_pending_ = true;
      E.perfc.incr(PC_adapt_device);
      return;
    }
    for (auto& a : async_in_) {  // could not start (previous buffers busy): the host adapts now
      AdaptState st = a.before;
      bool rearm = false;
      adapt_update(st, E.adapt_params, a.inst, a.miss, a.ssum, a.scnt, &rearm);
      async_apply(a.id, a.before, st);
    }
    async_in_.clear();
  }

  void dynamic_time_slice(int64_t now) {
    if (mode_ == Mode::ATC) update_acct_atc();
    E.timer_set(slice_ticker_, now + (int64_t)slice_period_us() * 1000);
  }
  uint32_t slice_period_us() const {
    return mode_ == Mode::ATC ? E.atc_params.apply_period_us : (uint32_t)E.boot.slice_apply_us;
  }

  void update_acct_atc() {
    uint32_t mn = 30000 * 10;
    std::vector<int> doms(active_sdom_.begin(), active_sdom_.end());
    for (int tid : doms) {
      CDom& d = sd(*E.tenants[tid]);
      atc_update(d.atc, E.atc_params);
      mn = std::min(mn, d.atc.tslice_us);
    }
    if (doms.empty()) return;
    atc_local_min_ = mn;
    // K11: the node-wide minimum from the other GPUs' pools (atc_sync), while fresh.
    if (atc_ext_min_ && E.now() < atc_ext_until_) mn = std::min(mn, atc_ext_min_);
    for (int tid : doms) {
      CDom& d = sd(*E.tenants[tid]);
      d.atc.tslice_us = mn;
      d.atc.hist[3].tslice = mn;
    }
    tslice_us_ = mn;
    recompute();
    E.perfc.incr(PC_atc_apply);
    E.emit(TRC_ATC, master_, mn, (uint32_t)doms.size());
  }

  // ATC across GPUs: the reference applies the minimum slice of
  // all domains every 21 ms; with one engine per GPU, the ranks MIN-reduce
  // their local minima (parallel/gang.py) and apply the node-wide one here.
  // Returns the local minimum of the last apply; a fresh global minimum is
  // applied at once and folded into the next applies for 3 periods.
  int atc_sync(int global_min_us) override {
    if (mode_ != Mode::ATC) return GPBS_EINVAL;
    if (global_min_us > 0) {
      atc_ext_min_ = (uint32_t)global_min_us;
      atc_ext_until_ = E.now() + 3 * (int64_t)slice_period_us() * 1000;
      if (atc_ext_min_ < tslice_us_) {
        for (int tid : active_sdom_) {
          CDom& d = sd(*E.tenants[tid]);
          d.atc.tslice_us = atc_ext_min_;
          d.atc.hist[3].tslice = atc_ext_min_;
        }
        tslice_us_ = atc_ext_min_;
        recompute();
        E.emit(TRC_ATC, master_, atc_ext_min_, (uint32_t)active_sdom_.size());
      }
    }
    return (int)(atc_local_min_ ? atc_local_min_ : tslice_us_);
  }

  // ----------------------------------------------------- wake / sleep ----
  void sleep(Slot& v) override {
    E.perfc.incr(PC_vcpu_sleep);
    sv(v).req_until = 0;
    if (E.parts[v.processor]->curr == v.id)
      E.raise_softirq(v.processor);
    else if (sv(v).runq_cpu >= 0)
      runq_remove(v);
  }

  void wake(Slot& v) override {
    CSlot& s = sv(v);
    if (E.parts[v.processor]->curr == v.id) {
      E.perfc.incr(PC_vcpu_wake_running);
      return;
    }
    if (s.runq_cpu >= 0) {
      E.perfc.incr(PC_vcpu_wake_onrunq);
      return;
    }
    E.perfc.incr(E.runnable(v) ? PC_vcpu_wake_runnable : PC_vcpu_wake_not_runnable);
    // Budget layout: a slot that blocked outside its budget (it ran there
    // before a relayout, or was stolen there) wakes at its class home -- it
    // is on no runqueue, so the move is free.  Otherwise a short-request
    // tenant (the slo mix's in-region latency tenant, blocked at every class
    // tick, so never sent home) kept waking on a GEMM's shader engine and
    // BOOST-preempted it at every request (round 6: the equal-quantum
    // ablations ran it on SE0/SE1 + SE3, GEMM 0.48 instead of 0.53).
    if (v.class_home >= 0 && !v.soft.empty() && !v.soft.test(v.processor) && v.affinity.test(v.class_home) &&
        E.pools[E.tenants[v.tenant]->pool]->cpus.test(v.class_home)) {
      const int from = v.processor;
      v.processor = v.class_home;
      v.homed_at = E.now();
      E.perfc.incr(PC_wake_homed);
      E.emit(TRC_MIGRATE, v.processor, v.tenant, v.index, from, v.processor);
    }
    if (s.pri == PRI_UNDER && !(s.flags & FLAG_PARKED)) {
      s.pri = PRI_BOOST;  // wake-boost
      s.req_until = E.now() + kReqWindowNs;
    }
    runq_insert(v.processor, v);
    tickle(v.processor, v);
  }

  uint32_t trace_word(Slot& v) override {
    if (!v.priv) return 0;
    const CSlot& s = sv(v);
    const int32_t c = std::max<int32_t>(-(1 << 23), std::min<int32_t>((1 << 23) - 1, s.credit));
    return (uint32_t)(s.pri + 128) & 0xffu | ((uint32_t)c << 8);
  }

  void yield(Slot& v) override {
    if (!E.boot.default_yield) sv(v).flags |= FLAG_YIELD;
  }

  // Report kinds (GPBS_REPORT_*): 1 wait (the vcrd_op spin report, P2),
  // 2 lock hold time (P8's prepared spinstat_op(holdtime, 2),
  // L:kernel/lockdep.c:3754-3759 -- tracked, not fed to adaptation, as in the
  // reference where the hook stayed commented out), 3 request arrivals (P7:
  // `wait` carries the count, the event-channel port-44 counter of
  // X:xen/common/event_channel.c:637-649 made live).
  void report(Tenant& d, uint64_t wait, int kind) override {
    CDom& s = sd(d);
    if (kind == GPBS_REPORT_HOLD) {
      s.lock_hold_ns += wait;
      s.lock_hold_count++;
      s.report_total++;
      return;
    }
    if (kind == GPBS_REPORT_REQUESTS) {
      d.pending_requests += wait;
      s.report_total++;
      return;
    }
    if (mode_ == Mode::ATC) {
      atc_report(s.atc, E.atc_params, wait);
      s.spinlock_latency += wait;  // cumulative, for introspection / gang decisions
    } else {  // do_vcrd_op (:249-259)
      s.spinlock_latency += wait;
      s.spinlock_metric_update += wait;
      s.spinlock_count++;
    }
    s.report_total++;
  }

  // -------------------------------------------------------- dispatch ----
  Slot* runq_steal(int peer, int cpu, int pri, bool soft_pass) {
    Slot& peer_cur = curr(peer);
    if (E.parts[peer]->priv && !peer_cur.is_idle()) {
      auto& rq = pc(peer).runq;
      for (int sid : rq) {
        Slot& v = *E.slots[sid];
        CSlot& s = sv(v);
        if (s.pri <= pri) break;
        if (v.is_idle()) continue;
        bool hot = (E.now() - v.last_run_time) < (int64_t)E.boot.migration_delay_us * 1000;
        if (hot) E.perfc.incr(PC_vcpu_hot);
        if (soft_pass && !v.soft.empty() && !v.soft.test(cpu)) continue;
        if (xgang(v, E.now()) == 2) continue;
        // A slot just sent to its class home is not stolen back across classes
        // for a while: every class migration briefly leaves the partition it
        // came from idle, and that partition would otherwise take the slot
        // straight back (the cache-hot guard of Xen's migration_delay, applied
        // to class placement).
        if (!soft_pass && !v.soft.empty() && !v.soft.test(cpu) &&
            E.now() - v.homed_at < std::max<int64_t>(1000000, 4 * (int64_t)ratelimit_us_ * 1000))
          continue;
        // (gpbs extension of csched_runq_steal, X:xen/common/sched_credit.c:1560-1605.)
        // Budget layout, time-shared class region: every tenant of the region
        // has a home slot on every partition of it, so a steal onto a
        // partition that already holds a runnable sibling of the slot only
        // stacks the tenant there and leaves a hole at the peer -- zero-sum
        // for the tenant's share, and the class tick then sends it home
        // (sleep + migrate + wake, a revocation of the runner's SEs each).
        // 8mix traces: ~1900 such steals per GEMM tenant per run in the slow
        // mode (0.68-1.00) vs ~500 in the fast one (1.13-1.17).
        if (E.boot.class_budget && E.boot.class_split > 1 && !E.boot.sibling_steal && sibling_on(cpu, v)) {
          E.perfc.incr(PC_steal_sibling_skip);
          continue;
        }
        if (!v.is_running && !hot && v.affinity.test(cpu)) {
          s.stats.migrate_q++;
          E.perfc.incr(PC_migrate_queued);
          runq_remove(v);
          int from = v.processor;
          v.processor = cpu;
          E.emit(TRC_STEAL, cpu, v.tenant, v.index, from, cpu);
          return &v;
        }
      }
    }
    E.perfc.incr(PC_steal_peer_idle);
    return nullptr;
  }

  Slot& load_balance(int cpu, Slot& snext, bool* stolen) {
    CSlot& s = sv(snext);
    if (s.pri == PRI_IDLE)
      E.perfc.incr(PC_load_balance_idle);
    else if (s.pri == PRI_OVER)
      E.perfc.incr(PC_load_balance_over);
    else
      E.perfc.incr(PC_load_balance_other);
    // Two balance steps (Xen 4.5's soft-affinity form of csched_load_balance,
    // X:xen/common/sched_credit.c:1607-1672 in 4.2.1): slots whose soft
    // affinity includes this partition first; then, only for an otherwise
    // idle partition, any slot hard affinity allows (cross-class work
    // conservation; off in the budget layout with boot class_steal=0).
    for (int step = 0; step < 2; ++step) {
      if (step == 1 && (s.pri != PRI_IDLE ||
                        (E.boot.class_budget && E.boot.class_split > 1 && !E.boot.class_steal)))
        break;
      Mask workers = online().andnot(idlers_);
      workers.clear(cpu);
      int peer = cpu;
      while (!workers.empty()) {
        peer = workers.cycle(peer);
        workers.clear(peer);
        // Single-dispatcher design: the peer's runqueue is always lockable.
        Slot* sp = runq_steal(peer, cpu, s.pri, step == 0);
        if (sp) {
          *stolen = true;
          return *sp;
        }
      }
    }
    runq_remove(snext);
    return snext;
  }

  // Contention-aware sibling selection (gpbs extension of _csched_cpu_pick's
  // SMT awareness): the two issue contexts of an XCD run concurrently and
  // share its CUs, L2 and the HBM path.  Among runnable slots of the head's
  // priority class, prefer one whose tenant is not memory-bound when a sibling
  // context already runs a memory-bound tenant (PBS miss-rate classification),
  // and never double-book a tenant on both contexts of one XCD.
  bool mem_bound(int tenant) {
    if (tenant < 0) return false;
    Tenant* t = E.tenant(tenant);
    return t && t->priv && sd(*t).rate_ewma >= E.adapt_params.threshold;
  }
  int conflict(const Slot& v, int cpu) {
    int score = 0;
    const Partition& P = *E.parts[cpu];
    for (int c = cpus_.first(); c >= 0; c = cpus_.next(c + 1)) {
      if (c == cpu) continue;
      const Partition& Q = *E.parts[c];
      if (Q.gpu != P.gpu || Q.xcd != P.xcd) continue;
      const int st = E.slots[Q.curr]->tenant;
      if (st < 0) continue;
      if (st == v.tenant)
        score += 2;
      else if (mem_bound(st) && mem_bound(v.tenant))
        score += 1;
    }
    return score;
  }
  Slot* cosched_pick(int cpu) {
    // SE-exclusive partitions share no issue slots: nothing to de-conflict,
    // and a tenant on several SEs of one XCD is the intended layout.
    if (E.boot.class_split > 1) return nullptr;
    auto& rq = pc(cpu).runq;
    Slot& head = *E.slots[rq.front()];
    const int16_t pri0 = sv(head).pri;
    int best_score = conflict(head, cpu);
    if (best_score == 0) return nullptr;
    Slot* best = nullptr;
    for (int sid : rq) {
      Slot& v = *E.slots[sid];
      if (sv(v).pri != pri0) break;
      if (v.is_idle()) continue;
      int s = conflict(v, cpu);
      if (s < best_score) {
        best_score = s;
        best = &v;
        if (s == 0) break;
      }
    }
    return best;
  }

  // Gang alignment (coschedule >= 3; Ousterhout co-scheduling applied to the
  // XCD partitions of one GPU): the partitions of one issue-context class on a
  // GPU form a gang led by its lowest-numbered partition.  The leader decides
  // by credit as usual; followers run the leader's tenant whenever they hold a
  // runnable slot of it, and are re-scheduled at once when the leader switches.
  // A memory-bound tenant then owns the whole HBM path for its quantum instead
  // of several bandwidth tenants each driving a few XCDs (per-CU load paths
  // cap what a partial-GPU tenant can pull, and their mixed streams thrash the
  // MALL), while credit keeps the shares fair over time.
  // With class_split > 1 (SE-exclusive mode) a gang is a whole class group
  // (all compute-class or all memory-class shader engines of the GPU), so a
  // memory tenant gets every memory SE for its quantum instead of sharing
  // them SE by SE with another memory tenant (per-CU load paths cap what one
  // SE can pull: profiles/se_interfere_1gpu.jsonl).
  int gang_key(int ctx) const {
    const int split = E.boot.class_split;
    return split > 1 ? (ctx < split ? 0 : 1) : ctx;
  }
  int gang_leader(int cpu) const {
    const Partition& P = *E.parts[cpu];
    for (int c = cpus_.first(); c >= 0; c = cpus_.next(c + 1)) {
      const Partition& Q = *E.parts[c];
      if (Q.gpu == P.gpu && gang_key(Q.ctx) == gang_key(P.ctx)) return c;
    }
    return cpu;
  }
  Slot* gang_pick(int cpu, Slot& head) {
    const int lead = gang_leader(cpu);
    if (lead == cpu) return nullptr;
    const int L = E.slots[E.parts[lead]->curr]->tenant;
    if (L < 0 || head.tenant == L) return nullptr;
    if (Tenant* lt = E.tenant(L); lt && lt->gang(E.now()) == 2) return nullptr;  // leader not yet rescheduled
    const int16_t hp = sv(head).pri;
    for (int sid : pc(cpu).runq) {
      Slot& v = *E.slots[sid];
      if (v.tenant != L) continue;
      const int16_t p = sv(v).pri;
      if (p < PRI_OVER) return nullptr;              // parked/idle
      if (hp > PRI_UNDER && p < hp) return nullptr;  // never delay a BOOSTed waker
      return &v;
    }
    return nullptr;
  }
  void gang_kick(int cpu) {
    const Partition& P = *E.parts[cpu];
    for (int c = cpus_.first(); c >= 0; c = cpus_.next(c + 1)) {
      if (c == cpu) continue;
      const Partition& Q = *E.parts[c];
      if (Q.gpu == P.gpu && gang_key(Q.ctx) == gang_key(P.ctx)) E.raise_softirq(c);
    }
  }
  bool gang_misaligned(int cpu, const Slot& scurr) {
    if (E.boot.coschedule < 3 || scurr.is_idle()) return false;
    const int lead = gang_leader(cpu);
    if (lead == cpu) return false;
    const int L = E.slots[E.parts[lead]->curr]->tenant;
    if (L < 0 || L == scurr.tenant) return false;
    for (int sid : pc(cpu).runq)
      if (E.slots[sid]->tenant == L) return true;
    return false;
  }

  // Cross-GPU gang windows (gpbs_gang_set, driven by parallel/gang.py): a
  // favoured tenant runs on every partition holding one of its runnable
  // slots (BOOSTed wakers of other tenants still preempt); an excluded one is
  // passed over and never stolen, so a collective's ranks on different GPUs
  // only run together.
  int xgang(const Slot& v, int64_t now) {
    if (v.is_idle()) return 0;
    Tenant* t = E.tenant(v.tenant);
    return t ? t->gang(now) : 0;
  }
  Slot* xgang_favoured(int cpu, Slot& head, int64_t now) {
    if (xgang(head, now) == 1) return nullptr;
    const int16_t hp = sv(head).pri;
    for (int sid : pc(cpu).runq) {
      Slot& v = *E.slots[sid];
      if (v.is_idle() || xgang(v, now) != 1) continue;
      const int16_t p = sv(v).pri;
      if (p < PRI_OVER) return nullptr;
      if (hp > PRI_UNDER && p < hp) return nullptr;
      return &v;
    }
    return nullptr;
  }
  Slot* xgang_first_allowed(int cpu, int64_t now) {
    for (int sid : pc(cpu).runq)
      if (xgang(*E.slots[sid], now) != 2) return E.slots[sid].get();
    return nullptr;
  }

  // BOOST exclusion (boost_exclusive; gpbs extension, no reference
  // counterpart): while a sibling context of this XCD runs a request -- a
  // slot inside the window opened by a BOOSTing wake (credit demotes BOOST at
  // its first accounting tick, long before a request ends, so the window is
  // tracked separately: it closes when the slot blocks, or after
  // kReqWindowNs for a tenant that never does) -- a memory-class slot of
  // another tenant parks instead of running, so the request gets the XCD's
  // share of HBM to itself.  The bytes the parked tenant would have moved in
  // that window are the ones the request moves instead, so throughput
  // tenants lose ~nothing while the request finishes near its solo latency.
  static constexpr int64_t kReqWindowNs = 1000000;
  bool in_request(Slot& v, int64_t now) { return !v.is_idle() && sv(v).req_until > now; }
  bool boost_excluded(int cpu, Slot& v) {
    if (!E.boot.boost_exclusive || v.is_idle() || !mem_bound(v.tenant)) return false;
    const int64_t now = E.now();
    if (in_request(v, now)) return false;
    const Partition& P = *E.parts[cpu];
    for (int c = cpus_.first(); c >= 0; c = cpus_.next(c + 1)) {
      if (c == cpu) continue;
      const Partition& Q = *E.parts[c];
      if (Q.gpu != P.gpu || Q.xcd != P.xcd) continue;
      Slot& o = *E.slots[Q.curr];
      if (o.tenant != v.tenant && in_request(o, now)) return true;
    }
    return false;
  }
  void kick_xcd(int cpu) {
    const Partition& P = *E.parts[cpu];
    for (int c = cpus_.first(); c >= 0; c = cpus_.next(c + 1))
      if (c != cpu && E.parts[c]->gpu == P.gpu && E.parts[c]->xcd == P.xcd) E.raise_softirq(c);
  }

  // Region virtual time (boot region_vt; gpbs extension).  In a time-shared
  // class region the co-sharers' credit cannot order them: the pool's fair
  // share of a slot (a whole partition per weight share) exceeds what a
  // crowded region can give, so every co-sharer sits at the credit ceiling,
  // UNDER, and the runqueue order alone rotates them -- one turn each, so a
  // tenant's share would follow its quantum.  Instead the region keeps the
  // partition-time each tenant ran there (per weight) and the next turn goes
  // to the least-served runnable co-sharer (a BOOSTed waker still first).
  // Per-tenant quanta then set how often a tenant switches, not its share.
  // A tenant that returns from an absence is lifted to the region's floor
  // minus two long quanta, so it cannot monopolise the region to catch up.
  int64_t rvt_floor_[2] = {0, 0};
  int64_t rvt_lag() const {
    return 2 * (int64_t)std::max<uint32_t>({E.adapt_params.max_us, tslice_us_,
                                            (uint32_t)std::max(0, E.boot.shared_q_us),
                                            (uint32_t)std::max(0, E.boot.switch_floor_max_us)}) * 1000;
  }
  void rvt_account(int cpu, Slot& cur, int64_t now) {
    CPcpu& p = pc(cpu);
    if (cur.is_idle() || !E.boot.region_vt) {
      p.rvt_mark = now;
      return;
    }
    Tenant& t = *E.tenants[cur.tenant];
    const int64_t from = std::max(p.rvt_mark, cur.rs_entry);
    p.rvt_mark = now;
    if (!shared_region(t) || now <= from) return;
    CDom& d = sd(t);
    d.rvt += (now - from) * 256 / std::max<int64_t>(1, d.weight);
  }
  Slot* region_pick(int cpu, Slot& head, int64_t now) {
    if (!E.boot.region_vt || head.is_idle() || sv(head).pri == PRI_BOOST) return nullptr;
    Tenant& ht = *E.tenants[head.tenant];
    if (!shared_region(ht)) return nullptr;
    const int rc = region_cls(ht) & 1;
    const int64_t lag = rvt_lag();
    Slot* best = nullptr;
    int64_t bv = 0;
    for (int sid : pc(cpu).runq) {
      Slot& v = *E.slots[sid];
      if (v.is_idle()) continue;
      const int16_t p = sv(v).pri;
      if (p == PRI_BOOST) return nullptr;  // a waker goes first (the runq head)
      if (p < PRI_OVER || xgang(v, now) == 2) continue;
      Tenant& t = *E.tenants[v.tenant];
      if (!cosharer(ht, t)) continue;
      CDom& d = sd(t);
      if (d.rvt < rvt_floor_[rc] - lag) d.rvt = rvt_floor_[rc] - lag;
      if (!best || d.rvt < bv) {
        best = &v;
        bv = d.rvt;
      }
    }
    if (best) rvt_floor_[rc] = std::max(rvt_floor_[rc], bv);
    return best == &head ? nullptr : best;
  }

  TaskSlice do_schedule(int cpu, int64_t now) override {
    Slot& scurr = curr(cpu);
    CSlot& cs = sv(scurr);
    const bool was_req = in_request(scurr, now) || (!scurr.is_idle() && !E.runnable(scurr));
    E.perfc.incr(PC_schedule);
    rvt_account(cpu, scurr, now);
    int64_t runtime = now - scurr.rs_entry;
    if (runtime < 0) runtime = 0;
    if (!scurr.is_idle()) {
      burn_credits(scurr, now);
      cs.start_time -= now;
    } else {
      cs.pri = PRI_IDLE;
    }
    Slot* snext = nullptr;
    TaskSlice ret{0, 0, false};
    int64_t tslice;
    bool held = false, parked = false;
    const int prev_tenant = scurr.tenant;
    if (ratelimit_us_ && E.runnable(scurr) && !scurr.is_idle() && runtime < (int64_t)ratelimit_us_ * 1000 &&
        !gang_misaligned(cpu, scurr) && xgang(scurr, now) != 2 && !xgang_favoured(cpu, scurr, now) &&
        !boost_excluded(cpu, scurr)) {
      snext = &scurr;
      cs.start_time += now;
      E.perfc.incr(PC_delay_ms);
      E.perfc.incr(PC_ratelimit_hold);
      tslice = (int64_t)ratelimit_us_ * 1000;
      held = true;
    } else {
      tslice = (int64_t)tslice_us_ * 1000;
      if (E.runnable(scurr)) runq_insert(cpu, scurr);
      auto& rq = pc(cpu).runq;
      snext = E.slots[rq.front()].get();
      bool follow = false;
      if (Slot* f = xgang_favoured(cpu, *snext, now)) {
        rq.remove(f->id);
        rq.push_front(f->id);
        snext = f;
        follow = true;
      } else if (xgang(*snext, now) == 2) {
        if (Slot* a = xgang_first_allowed(cpu, now)) {
          rq.remove(a->id);
          rq.push_front(a->id);
          snext = a;
        }
      }
      if (!follow && E.boot.coschedule >= 3) {
        if (Slot* g = gang_pick(cpu, *snext)) {
          rq.remove(g->id);
          rq.push_front(g->id);
          snext = g;
          follow = true;
        }
      }
      if (!follow) {
        if (Slot* r = region_pick(cpu, *snext, now)) {  // least-served co-sharer of a time-shared region
          rq.remove(r->id);
          rq.push_front(r->id);
          snext = r;
          follow = true;  // picked by region time, not by credit priority: no steal
        }
      }
      if (!follow && E.boot.coschedule && !snext->is_idle()) {
        Slot* alt = cosched_pick(cpu);
        if (alt && xgang(*alt, now) != 2) {  // same priority class, less contention
          rq.remove(alt->id);
          rq.push_front(alt->id);
          snext = alt;
        }
      }
      if (cs.flags & FLAG_YIELD) cs.flags &= ~FLAG_YIELD;
      if (sv(*snext).pri > PRI_OVER || follow)
        runq_remove(*snext);
      else
        snext = &load_balance(cpu, *snext, &ret.migrated);
      if (boost_excluded(cpu, *snext)) {  // park behind the sibling's request
        runq_insert(cpu, *snext);
        snext = E.slots[E.parts[cpu]->idle_slot].get();
        parked = true;
        E.perfc.incr(PC_boost_park);
      }
      if (sv(*snext).pri == PRI_IDLE && !parked)
        idlers_.set(cpu);
      else
        idlers_.clear(cpu);
      if (!snext->is_idle()) sv(*snext).start_time += now;
    }
    // PBS (:1796-1804): the quantum is the next tenant's private tslice.
    // Q13: the reference applies this at `out:` (:1792-1797), *after* the
    // ratelimit hold of :1732, so a slot kept for ratelimit gets its whole
    // adaptive quantum (up to 1.1 ms there, 11 ms in the MI355X profile) and a
    // BOOSTed waker that tickled it waits that long.  gpbs holds for the
    // remaining ratelimit only (Xen >= 4.3 semantics); strict_ref keeps the
    // reference behaviour.
    if (held && !E.adapt_params.strict_ref) {
      tslice = std::max<int64_t>((int64_t)ratelimit_us_ * 1000 - runtime, 1000);
    } else if (!snext->is_idle()) {
      // per-tenant quantum (PBS :1796-1804; classq; the global slice of
      // credit-fixed and atc :1916), with the region floors / caps
      Tenant& nt = *E.tenants[snext->tenant];
      const uint32_t q = quantum_us(nt);
      tslice = (int64_t)q * 1000;
      if (!held) sd(nt).q_disp_us = q;
    } else {
      tslice = (int64_t)tslice_us_ * 1000;
    }
    // Measurement tenure (hardware counters): the first tenure that starts
    // after the sampler's request runs at least the requested length, once.
    // Credit still charges every microsecond of it, so the tenant's share
    // is unchanged over a few accounting periods.
    if (snext != &scurr && !snext->is_idle() && !held) {
      Tenant& tn = *E.tenants[snext->tenant];
      if (tn.measure_us) {
        tslice = std::max<int64_t>(tslice, (int64_t)tn.measure_us * 1000);
        tn.measure_us = 0;
        tn.measure_granted++;
      }
    }
    // A parked partition re-checks at least every 200 us (the request may
    // lose BOOST while still running, which kicks nobody).
    ret.time_ns = parked ? 200000 : (snext->is_idle() ? -1 : tslice);
    ret.slot = snext->id;
    if (E.boot.boost_exclusive && snext != &scurr &&
        (was_req || in_request(*snext, now)))
      kick_xcd(cpu);
    if (E.boot.coschedule >= 3 && snext->tenant != prev_tenant && !snext->is_idle() && gang_leader(cpu) == cpu)
      gang_kick(cpu);
    return ret;
  }

  // --------------------------------------------------------- control ----
  int adjust(Tenant& dom, bool set, int* weight, int* cap) override {
    CDom& d = sd(dom);
    if (!set) {
      *weight = d.weight;
      *cap = d.cap;
      return 0;
    }
    if (*weight != -1 && *weight != 0) {
      if (*weight < 1 || *weight > GPBS_WEIGHT_MAX) return GPBS_ERANGE;
      if (d.on_active) {
        weight_ -= (uint32_t)d.weight * d.active_vcpu_count;
        weight_ += (uint32_t)*weight * d.active_vcpu_count;
      }
      d.weight = (uint16_t)*weight;
    }
    if (*cap != -1) {
      if (*cap < 0 || *cap > 100 * (int)dom.slots.size()) return GPBS_ERANGE;
      d.cap = (uint16_t)*cap;
    }
    return 0;
  }

  int adjust_global(bool set, int* tslice_us, int* ratelimit_us) override {
    if (set) {
      if (*tslice_us > GPBS_TSLICE_UMAX || *tslice_us < GPBS_TSLICE_UMIN || *ratelimit_us > GPBS_RATELIMIT_MAX ||
          (*ratelimit_us < GPBS_RATELIMIT_MIN && *ratelimit_us != 0) || *ratelimit_us > *tslice_us)
        return GPBS_EINVAL;
      tslice_us_ = (uint32_t)*tslice_us;
      ratelimit_us_ = (uint32_t)*ratelimit_us;
      recompute();  // Q2 fix
      if (mode_ == Mode::FIXED)
        for (auto& t : E.tenants)
          if (t && t->alive && t->pool == pool_ && t->priv) {
            sd(*t).adapt.tslice_us = tslice_us_;
            sd(*t).adapt.tick_period_us = tick_period_us_;
          }
    }
    *tslice_us = (int)tslice_us_;
    *ratelimit_us = (int)ratelimit_us_;
    return 0;
  }

  int classify(Tenant& t) override {
    CDom& d = sd(t);
    if (d.pmc[0] == 0) return -1;  // idle this period: keep the current class
    // +-25 % band around the threshold: a tenant whose smoothed miss rate
    // hovers near it (a decode step streaming weights next to its attention,
    // a trainer's optimizer phase) keeps its class instead of flapping
    // between the class homes (each flip drains and re-homes its slots).
    const uint64_t thr = E.adapt_params.threshold;
    if (t.cls == 1) return d.rate_ewma >= thr * 3 / 4 ? 1 : 0;
    if (t.cls == 0) return d.rate_ewma >= thr * 5 / 4 ? 1 : 0;
    return d.rate_ewma >= thr ? 1 : 0;
  }

  // PBS with the gpbs detector extensions (grow_pct > 0): a confirmed class
  // change is a phase change the detector would otherwise find only after
  // refilling its window and climbing step by step -- with metric updates
  // once per clean counter window that is most of a 300 ms phase (phase-ts:
  // the phase tenant sat at min_us in 0.65 of its periods under gpbs, 0.54
  // under credit-classq).  Restart the detector from the new class's bound:
  // memory -> max_us, compute -> min_us, window re-armed.  Not at the first
  // classification: a jump of every tenant of a gang-switched region from
  // the initial quantum at once put the region out of step in simulation
  // (tests/test_se_mode.py), and the detector's own climb is fine there.
  void class_changed(Tenant& t, int from, int to) override {
    if (mode_ != Mode::PBS || !E.adapt_params.grow_pct || from < 0 || to < 0 || from == to) return;
    AdaptState& a = sd(t).adapt;
    a.tslice_us = to == 1 ? E.adapt_params.max_us : E.adapt_params.min_us;
    a.tick_period_us = a.tslice_us / std::max<uint32_t>(1, E.adapt_params.ticks_per_tslice);
    a.window_left = kWindow;
    a.stable_count = 0;
    for (auto& f : a.filter) f = FilterEntry{};
  }

  int bound_stats(Tenant& t, uint64_t* out3, bool reset) override {
    CDom& d = sd(t);
    if (out3) {
      out3[0] = d.bound_periods;
      out3[1] = d.bound_min;
      out3[2] = d.bound_max;
    }
    if (reset) d.bound_periods = d.bound_min = d.bound_max = 0;
    return 0;
  }

  bool tenant_adapt(Tenant& d, AdaptState* out) override {
    *out = sd(d).adapt;
    return true;
  }
  bool set_tenant_adapt(Tenant& d, const AdaptState& st) override {
    sd(d).adapt = st;
    return true;
  }

  void fill_tenant_info(Tenant& dom, gpbs_tenant_info_t& o) override {
    CDom& d = sd(dom);
    o.weight = d.weight;
    o.cap = d.cap;
    o.active_slots = d.active_vcpu_count;
    o.tslice_us = reported_us(dom);  // dispatched
    o.target_tslice_us = target_us(dom);
    o.last_dispatch_us = d.q_disp_us;
    o.tick_period_us = mode_ == Mode::PBS ? d.adapt.tick_period_us
                                          : (mode_ == Mode::CLASSQ ? o.target_tslice_us / E.adapt_params.ticks_per_tslice
                                                                   : tick_period_us_);
    o.phase = d.adapt.phase;
    o.window_left = d.adapt.window_left;
    o.last_err = d.adapt.last_err;
    o.last_curr = d.adapt.last_curr;
    o.last_win = d.adapt.last_win;
    for (int i = 0; i < 4; ++i) o.pmc[i] = d.pmc[i];
    o.cache_miss_rate = d.cache_miss_rate;
    o.cpi = d.cpi;
    o.spin_latency = d.spinlock_latency;
    o.report_count = d.report_total;
    o.pending_requests = d.pending_requests;
  }

  void fill_slot_info(Slot& v, gpbs_slot_info_t& o) override {
    CSlot& s = sv(v);
    o.pri = s.pri;
    o.flags = s.flags;
    o.credit = s.credit;
    o.on_runq = s.runq_cpu >= 0;
  }

  // ------------------------------------------------------------ dumps ----
  void dump_vcpu(Slot& v, std::string& o) {
    CSlot& s = sv(v);
    o += fmt("[%d.%d] pri=%d flags=%x cpu=%d", v.tenant, v.index, s.pri, s.flags, v.processor);
    if (!v.is_idle()) {
      o += fmt(" credit=%d [w=%u]", s.credit, sd_of(v).weight);
      o += fmt(" (%d+%u) {a/i=%u/%u m=%u+%u}", s.stats.credit_last, s.stats.credit_incr, s.stats.state_active,
               s.stats.state_idle, s.stats.migrate_q, s.stats.migrate_r);
    }
    o += "\n";
  }

  void dump_cpu_state(int cpu, std::string& o) override {
    CPcpu& p = pc(cpu);
    o += fmt(" sort=%u, sibling=%s, ", p.runq_sort_last, sibling_mask(cpu).str().c_str());
    o += fmt("core=%s\n", core_mask(cpu).str().c_str());
    o += "\trun: ";
    dump_vcpu(curr(cpu), o);
    int loop = 0;
    for (int sid : p.runq) {
      o += fmt("\t%3d: ", ++loop);
      dump_vcpu(*E.slots[sid], o);
    }
  }

  void dump_settings(std::string& o) override {
    o += fmt(
        "info:\n\tncpus              = %u\n\tmaster             = %d\n\tcredit             = %u\n"
        "\tcredit balance     = %d\n\tweight             = %u\n\trunq_sort          = %u\n"
        "\tdefault-weight     = %d\n\ttslice             = %uus\n\tratelimit          = %uus\n"
        "\tcredits per msec   = %d\n\tticks per tslice   = %u\n\tmigration delay    = %uus\n",
        ncpus_, master_, credit_, credit_balance_, weight_, runq_sort_, kDefaultWeight, tslice_us_, ratelimit_us_,
        1000, ticks_per_tslice_, (unsigned)E.boot.migration_delay_us);
    o += fmt("idlers: %s\n", idlers_.str().c_str());
    o += "active vcpus:\n";
    int loop = 0;
    for (int tid : active_sdom_)
      for (int sid : sd(*E.tenants[tid]).active_vcpu) {
        o += fmt("\t%3d: ", ++loop);
        dump_vcpu(*E.slots[sid], o);
      }
    o += "\n";
  }

  void dump_admin_conf(std::string& o) override {
    // csched_dump_customized (:1942-1974): cpus + per-slot pmuinfo/sched_count,
    // plus the live PBS state (quantum, phase, miss rate) per tenant.
    o += fmt("cpus: %s\n", cpus_.str().c_str());
    for (auto& t : E.tenants) {
      if (!t || !t->alive || t->pool != pool_ || !t->priv) continue;
      CDom& d = sd(*t);
      o += fmt("dom%d    (%s) tslice=%uus tick=%uus phase=%s miss_rate=%" PRIu64 " cpi=%" PRIu64
               " window_left=%u reports=%" PRIu64 "\n",
               t->id, t->name.c_str(), mode_ == Mode::PBS ? d.adapt.tslice_us : tslice_us_,
               mode_ == Mode::PBS ? d.adapt.tick_period_us : tick_period_us_,
               d.adapt.phase == kPhaseLow ? "LOW(cache-sensitive)" : "HIGH", d.cache_miss_rate, d.cpi,
               d.adapt.window_left, d.report_total);
      if (d.spinlock_count || d.lock_hold_count || t->pending_requests)
        o += fmt("    waits: n=%" PRIu64 " total=%" PRIu64 "ns  holds: n=%" PRIu64 " total=%" PRIu64
                 "ns  pending_requests=%" PRIu64 "\n",
                 d.spinlock_count, d.spinlock_latency, d.lock_hold_count, d.lock_hold_ns, t->pending_requests);
      for (int sid : t->slots) {
        Slot& v = *E.slots[sid];
        o += fmt("    vcpu%d: \n", v.index);
        o += fmt("        pmuinfo: INST_RETIRED=%" PRIu64 "  CPU_CLK_UNHALTED=%" PRIu64 "  LLC_REFERENCES=%" PRIu64
                 "  LLC_MISSES=%" PRIu64 "\n",
                 v.pmc[0], v.pmc[1], v.pmc[2], v.pmc[3]);
        o += fmt("        sched_count: %" PRIu64 "\n", v.sched_count);
      }
    }
    o += "\n";
  }

  std::string check() override {
    std::string err;
    uint64_t w = 0;
    for (int tid : active_sdom_) {
      CDom& d = sd(*E.tenants[tid]);
      if (d.active_vcpu_count != d.active_vcpu.size()) err += fmt("dom%d active count mismatch\n", tid);
      w += (uint64_t)d.weight * d.active_vcpu_count;
    }
    if (w != weight_) err += fmt("pool%d weight %u != sum %" PRIu64 "\n", pool_, weight_, w);
    for (int c = cpus_.first(); c >= 0; c = cpus_.next(c + 1)) {
      for (int sid : pc(c).runq) {
        Slot& v = *E.slots[sid];
        if (sv(v).runq_cpu != c) err += fmt("slot %d on runq %d but marks %d\n", sid, c, sv(v).runq_cpu);
        if (v.processor != c) err += fmt("slot %d on runq %d but processor %d\n", sid, c, v.processor);
        if (v.is_running) err += fmt("slot %d running and queued\n", sid);
      }
    }
    return err;
  }

 private:
  Mode mode_;
  std::list<int> active_sdom_;
  uint32_t ncpus_ = 0;
  int master_ = -1;
  int master_ticker_ = -1, slice_ticker_ = -1;
  Mask idlers_, cpus_;
  uint32_t weight_ = 0, credit_ = 0;
  int32_t credit_balance_ = 0;
  uint32_t runq_sort_ = 0;
  uint32_t ratelimit_us_ = 0, tslice_us_ = 0, tick_period_us_ = 0, ticks_per_tslice_ = 3, credits_per_tslice_ = 0;
  uint32_t atc_local_min_ = 0, atc_ext_min_ = 0;
  int64_t atc_ext_until_ = 0;
  int last_tickle_cpu_ = 0;
};

}  // namespace

std::unique_ptr<Scheduler> make_static_scheduler(Engine& e, int pool);
std::unique_ptr<Scheduler> make_credit2_scheduler(Engine& e, int pool);
std::unique_ptr<Scheduler> make_sedf_scheduler(Engine& e, int pool);
std::unique_ptr<Scheduler> make_arinc653_scheduler(Engine& e, int pool);

std::unique_ptr<Scheduler> make_scheduler(const std::string& name, Engine& e, int pool) {
  if (name == "credit" || name == "pbs") return std::make_unique<CreditScheduler>(e, pool, Mode::PBS);
  if (name == "credit-fixed") return std::make_unique<CreditScheduler>(e, pool, Mode::FIXED);
  if (name == "credit-classq") return std::make_unique<CreditScheduler>(e, pool, Mode::CLASSQ);
  if (name == "atc") return std::make_unique<CreditScheduler>(e, pool, Mode::ATC);
  if (name == "static") return make_static_scheduler(e, pool);
  if (name == "arinc653") return make_arinc653_scheduler(e, pool);
  if (name == "credit2") return make_credit2_scheduler(e, pool);
  if (name == "sedf") return make_sedf_scheduler(e, pool);
  return nullptr;
}

}  // namespace gpbs
