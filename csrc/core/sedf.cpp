// sedf: Simple Earliest Deadline First with slack ("extra time") sharing (S4).
//
// Behaviour parity with X:xen/common/sched_sedf.c (Xen 4.2).  Every slot has
// a (period, slice) reservation on its partition, or a weight that is turned
// into one (sedf_adjust_weights :1293-1366); tenants without a reservation are
// best effort and only run in extra time.
//   * per partition: an EDF run queue (sorted by absolute deadline), a wait
//     queue (sorted by the start of the next period), and two extra-time
//     queues -- L0 "penalty" (slots that lost slice to a short block) before
//     L1 "utilisation" (weighted round robin by score) (:28-43, :667-752);
//   * do_schedule: deschedule the current slot (EDF bookkeeping or extra-time
//     re-scoring, desched_edf_dom :406-468 / desched_extra_dom :561-665),
//     promote started periods / fix missed deadlines (update_queues :470-558),
//     then run the earliest deadline until its slice ends or the next period
//     begins, else extra time in EXTRA_QUANTUM pieces, else idle
//     (sedf_do_schedule :754-858);
//   * wake: a block inside the current period is a short block -- no more
//     real-time this period, the lost slice becomes L0 penalty score
//     (unblock_short_extra_support :955-1010); a longer block restarts the
//     period at the wake time, or with a latency hint, at a shortened period
//     whose slice doubles back each period (unblock_long_cons_b :1012-1019,
//     the 2c latency scaling in desched_edf_dom :424-436);
//   * should_switch (:1039-1083) decides whether a wake preempts.
// Slots are bound to their partition (sedf has no load balancing); placement
// cycles through the partitions the slot's affinity allows (sedf_pick_cpu).
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <list>

#include "engine.h"

namespace gpbs {
namespace {

constexpr int64_t kUs = 1000;
constexpr int64_t kMs = 1000 * kUs;
constexpr int64_t kExtraQuantum = 500 * kUs;     // EXTRA_QUANTUM
constexpr int64_t kWeightPeriod = 100 * kMs;     // WEIGHT_PERIOD
constexpr int64_t kWeightSafety = 5 * kMs;       // WEIGHT_SAFETY
constexpr int64_t kPeriodMax = 10000 * kMs;      // PERIOD_MAX
constexpr int64_t kPeriodMin = 10 * kUs;         // PERIOD_MIN
constexpr int64_t kSliceMin = 5 * kUs;           // SLICE_MIN
constexpr uint32_t EXTRA_AWARE = 1, EXTRA_RUN_PEN = 2, EXTRA_RUN_UTIL = 4, EXTRA_WANT_PEN_Q = 8, SEDF_ASLEEP = 16;
constexpr int PEN_Q = 0, UTIL_Q = 1;
enum QState { Q_NONE = 0, Q_RUN = 1, Q_WAIT = 2 };

std::string efmt(const char* f, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}

struct SedfSlot : SchedSlotData {
  int64_t period = kWeightPeriod, slice = 0, period_orig = kWeightPeriod, slice_orig = 0;
  int64_t latency = 0;
  int weight = 0, extraweight = 1;
  uint32_t status = EXTRA_AWARE | SEDF_ASLEEP;
  int64_t deadl_abs = 0, cputime = 0, sched_start_abs = 0, block_abs = 0;
  int64_t score[2] = {0, 0};
  int64_t short_block_lost_tot = 0, extra_time_tot = 0;
  uint64_t block_tot = 0, short_block_tot = 0, long_block_tot = 0, pen_extra_slices = 0, missed = 0;
  QState q = Q_NONE;
  bool on_extra[2] = {false, false};
  int64_t period_begin() const { return deadl_abs - period; }
};
struct SedfDom : SchedTenantData {  // xl-visible parameters, in us
  int64_t period = kWeightPeriod / kUs, slice = 0, latency = 0;
  int extratime = 1, weight = 0;
};
struct SedfPcpu : SchedPartData {
  std::list<int> runq, waitq, extraq[2];
  int64_t current_slice_expires = 0;
};

class SedfScheduler : public Scheduler {
 public:
  SedfScheduler(Engine& e, int pool) : Scheduler(e, pool) {}
  const char* name() const override { return "Simple EDF Scheduler"; }
  const char* opt_name() const override { return "sedf"; }

  SedfSlot& sv(Slot& v) { return *static_cast<SedfSlot*>(v.priv.get()); }
  SedfDom& sd(Tenant& d) { return *static_cast<SedfDom*>(d.priv.get()); }
  SedfPcpu& pc(int c) { return *static_cast<SedfPcpu*>(E.parts[c]->priv.get()); }
  bool has_pc(int c) { return c >= 0 && c < (int)E.parts.size() && E.parts[c]->priv; }

  // ------------------------------------------------------------ queues ---
  void del_from_queue(Slot& v) {
    SedfSlot& s = sv(v);
    if (s.q == Q_NONE || !has_pc(v.processor)) {
      s.q = Q_NONE;
      return;
    }
    (s.q == Q_RUN ? pc(v.processor).runq : pc(v.processor).waitq).remove(v.id);
    s.q = Q_NONE;
  }
  void add_sorted(std::list<int>& l, Slot& v, bool by_deadline) {
    const int64_t key = by_deadline ? sv(v).deadl_abs : sv(v).period_begin();
    auto it = l.begin();
    for (; it != l.end(); ++it) {
      SedfSlot& o = sv(*E.slots[*it]);
      if (key < (by_deadline ? o.deadl_abs : o.period_begin())) break;
    }
    l.insert(it, v.id);
  }
  void add_to_runq(Slot& v) {
    add_sorted(pc(v.processor).runq, v, true);
    sv(v).q = Q_RUN;
  }
  void add_to_waitq(Slot& v) {
    add_sorted(pc(v.processor).waitq, v, false);
    sv(v).q = Q_WAIT;
  }
  void extraq_del(Slot& v, int i) {
    if (!sv(v).on_extra[i]) return;
    if (has_pc(v.processor)) pc(v.processor).extraq[i].remove(v.id);
    sv(v).on_extra[i] = false;
  }
  // extraq_add_sort_update: every queued entry is charged `sub`, the slot is
  // inserted in score order (lower score = earlier extra time).
  void extraq_add_sort_update(Slot& v, int i, int64_t sub) {
    auto& l = pc(v.processor).extraq[i];
    auto pos = l.end();
    for (auto it = l.begin(); it != l.end(); ++it) {
      SedfSlot& o = sv(*E.slots[*it]);
      o.score[i] -= sub;
      if (pos == l.end() && sv(v).score[i] < o.score[i]) pos = it;
    }
    l.insert(pos, v.id);
    sv(v).on_extra[i] = true;
  }
  void extraq_check_add_unblocked(Slot& v) {
    if ((sv(v).status & EXTRA_AWARE) && !sv(v).on_extra[UTIL_Q]) extraq_add_sort_update(v, UTIL_Q, 0);
  }
  bool extra_runs(const SedfSlot& s) { return s.status & (EXTRA_RUN_PEN | EXTRA_RUN_UTIL); }

  // ---------------------------------------------------- deschedule -------
  void desched_edf(int64_t now, Slot& v) {
    SedfSlot& s = sv(v);
    s.cputime += now - s.sched_start_abs;
    const bool runnable = !(s.status & SEDF_ASLEEP);
    if (s.cputime < s.slice && runnable) return;
    del_from_queue(v);
    if (s.cputime >= s.slice) {
      s.cputime -= s.slice;
      if (s.period < s.period_orig) {  // latency scaling: grow back to the reservation
        s.period *= 2;
        s.slice *= 2;
        if (s.period > s.period_orig || s.slice > s.slice_orig) {
          s.period = s.period_orig;
          s.slice = s.slice_orig;
        }
      }
      s.deadl_abs += s.period;
    }
    if (runnable) {
      add_to_waitq(v);
    } else {
      extraq_del(v, PEN_Q);
      extraq_del(v, UTIL_Q);
    }
  }

  void desched_extra(int64_t now, Slot& v) {
    SedfSlot& s = sv(v);
    const int i = (s.status & EXTRA_RUN_PEN) ? PEN_Q : UTIL_Q;
    s.status &= ~(EXTRA_RUN_PEN | EXTRA_RUN_UTIL);
    s.cputime = 0;
    s.extra_time_tot += now - s.sched_start_abs;
    extraq_del(v, i);
    int64_t oldscore = s.score[i];
    if (i == PEN_Q) {
      // The block penalty is considered compensated after one extra run
      // (the reference's "#if 0" KAF note: otherwise one tenant can starve
      // the rest for seconds).
      s.short_block_lost_tot = 0;
      s.status &= ~EXTRA_WANT_PEN_Q;
    } else {
      s.score[UTIL_Q] = s.extraweight ? (int64_t(1) << 17) / s.extraweight
                                      : (s.slice > 0 ? (s.period << 10) / s.slice : (int64_t(1) << 17));
    }
    const bool runnable = !(s.status & SEDF_ASLEEP);
    if (runnable) {
      if (((s.status & EXTRA_AWARE) && i == UTIL_Q) || ((s.status & EXTRA_WANT_PEN_Q) && i == PEN_Q))
        extraq_add_sort_update(v, i, oldscore);
    } else {
      del_from_queue(v);
      extraq_del(v, i == PEN_Q ? UTIL_Q : PEN_Q);
    }
  }

  void update_queues(int64_t now, SedfPcpu& p) {
    while (!p.waitq.empty()) {
      Slot& v = *E.slots[p.waitq.front()];
      if (sv(v).period_begin() > now) break;
      del_from_queue(v);
      add_to_runq(v);
    }
    for (auto it = p.runq.begin(); it != p.runq.end();) {
      Slot& v = *E.slots[*it];
      SedfSlot& s = sv(v);
      ++it;
      if (s.slice == 0) {  // best effort: park in the waitq at the next period
        del_from_queue(v);
        s.deadl_abs += s.period;
        if (s.period_begin() < now) s.deadl_abs += (now - s.period_begin() + s.period - 1) / s.period * s.period;
        add_to_waitq(v);
      } else if (s.deadl_abs < now || s.cputime > s.slice) {  // missed deadline / overran
        s.missed++;
        del_from_queue(v);
        s.deadl_abs += s.period;
        if (s.deadl_abs < now) s.deadl_abs += (now - s.deadl_abs + s.period - 1) / s.period * s.period;
        s.cputime = 0;
        if (s.period_begin() > now)
          add_to_waitq(v);
        else
          add_to_runq(v);
      } else {
        break;
      }
    }
  }

  TaskSlice extra_schedule(int64_t now, int64_t end_xt, int cpu) {
    SedfPcpu& p = pc(cpu);
    if (end_xt - now >= kExtraQuantum) {
      for (int i : {PEN_Q, UTIL_Q}) {
        if (p.extraq[i].empty()) continue;
        Slot& v = *E.slots[p.extraq[i].front()];
        sv(v).status |= (i == PEN_Q ? EXTRA_RUN_PEN : EXTRA_RUN_UTIL);
        if (i == PEN_Q) sv(v).pen_extra_slices++;
        return TaskSlice{v.id, kExtraQuantum, false};
      }
    }
    return TaskSlice{E.parts[cpu]->idle_slot, std::max<int64_t>(end_xt - now, kUs), false};
  }

  TaskSlice do_schedule(int cpu, int64_t now) override {
    E.perfc.incr(PC_schedule);
    SedfPcpu& p = pc(cpu);
    Slot& cur = E.curr_of(cpu);
    if (!cur.is_idle() && cur.priv) {
      SedfSlot& s = sv(cur);
      if (!E.runnable(cur)) s.status |= SEDF_ASLEEP;
      if (s.status & SEDF_ASLEEP) s.block_abs = now;
      if (extra_runs(s))
        desched_extra(now, cur);
      else
        desched_edf(now, cur);
    }
    update_queues(now, p);
    TaskSlice ret{E.parts[cpu]->idle_slot, -1, false};
    if (p.runq.empty() && p.waitq.empty()) {
      ret.time_ns = -1;
    } else if (!p.runq.empty()) {
      Slot& r = *E.slots[p.runq.front()];
      ret.slot = r.id;
      int64_t t = sv(r).slice - sv(r).cputime;
      if (!p.waitq.empty()) t = std::min(now + t, sv(*E.slots[p.waitq.front()]).period_begin()) - now;
      ret.time_ns = t;
    } else {
      ret = extra_schedule(now, sv(*E.slots[p.waitq.front()]).period_begin(), cpu);
    }
    if (ret.time_ns == 0 || (ret.time_ns < 0 && ret.slot != E.parts[cpu]->idle_slot))
      ret.time_ns = kExtraQuantum;  // "seriously BEHIND schedule"
    Slot& n = *E.slots[ret.slot];
    if (!n.is_idle()) {
      sv(n).sched_start_abs = now;
      if (n.processor != cpu) n.processor = cpu;
    }
    p.current_slice_expires = ret.time_ns >= 0 ? now + ret.time_ns : INT64_MAX;
    return ret;
  }

  // ------------------------------------------------------ wake / sleep ---
  void sleep(Slot& v) override {
    E.perfc.incr(PC_vcpu_sleep);
    sv(v).status |= SEDF_ASLEEP;
    if (E.parts[v.processor]->curr == v.id) {
      E.raise_softirq(v.processor);
    } else {
      del_from_queue(v);
      extraq_del(v, UTIL_Q);
      extraq_del(v, PEN_Q);
    }
  }

  int run_type(Slot& v) {
    if (v.is_idle()) return 4;
    if (sv(v).status & EXTRA_RUN_PEN) return 2;
    if (sv(v).status & EXTRA_RUN_UTIL) return 3;
    return 1;
  }
  bool should_switch(Slot& cur, Slot& other) {
    SedfSlot& o = sv(other);
    if (has_pc(other.processor) && o.period_begin() < pc(other.processor).current_slice_expires) return true;
    switch (run_type(cur)) {
      case 1: return false;
      case 2: return (o.status & EXTRA_WANT_PEN_Q) && o.score[PEN_Q] < sv(cur).score[PEN_Q];
      case 3: return (o.status & EXTRA_WANT_PEN_Q) != 0;
      default: return true;
    }
  }

  void wake(Slot& v) override {
    if (E.parts[v.processor]->curr == v.id) {
      sv(v).status &= ~SEDF_ASLEEP;
      E.perfc.incr(PC_vcpu_wake_running);
      return;
    }
    SedfSlot& s = sv(v);
    if (s.q != Q_NONE) {
      E.perfc.incr(PC_vcpu_wake_onrunq);
      return;
    }
    if (!has_pc(v.processor) || !v.affinity.test(v.processor)) v.processor = pick_cpu(v);
    if (!has_pc(v.processor)) return;
    E.perfc.incr(PC_vcpu_wake_runnable);
    const int64_t now = E.now();
    s.status &= ~SEDF_ASLEEP;
    if (s.deadl_abs == 0) s.deadl_abs = now + s.slice;  // initial deadline
    s.block_tot++;
    if (now < s.period_begin()) {  // woke in extra time
      if ((s.status & EXTRA_WANT_PEN_Q) && !s.on_extra[PEN_Q]) extraq_add_sort_update(v, PEN_Q, 0);
      extraq_check_add_unblocked(v);
    } else if (now < s.deadl_abs) {  // short block
      s.short_block_tot++;
      s.deadl_abs += s.period;  // no more real time this period
      int64_t pen = std::max<int64_t>(0, s.slice - s.cputime);
      s.short_block_lost_tot = pen;
      if (pen) {
        s.score[PEN_Q] = (s.period << 10) / pen;
        if (s.on_extra[PEN_Q])
          extraq_del(v, PEN_Q);
        else
          s.status |= EXTRA_WANT_PEN_Q;
        extraq_add_sort_update(v, PEN_Q, 0);
      }
      s.cputime = 0;
      extraq_check_add_unblocked(v);
    } else {  // long block: new period from now (2b), latency-scaled (2c)
      s.long_block_tot++;
      if (s.latency > 0 && s.slice_orig > 0 && s.latency < s.period_orig) {
        s.period = s.latency;
        s.slice = std::max<int64_t>(kSliceMin, s.slice_orig * s.latency / s.period_orig);
      }
      s.deadl_abs = now + s.period;
      s.cputime = 0;
      extraq_check_add_unblocked(v);
    }
    if (s.period_begin() > now)
      add_to_waitq(v);
    else
      add_to_runq(v);
    if (should_switch(E.curr_of(v.processor), v)) E.raise_softirq(v.processor);
  }
  void yield(Slot&) override {}

  int pick_cpu(Slot& v) override {
    const Mask ok = E.pools[pool_]->cpus & v.affinity;
    if (ok.empty()) return E.pools[pool_]->cpus.first();
    const int c = ok.cycle(v.processor);
    return c >= 0 ? c : ok.first();
  }

  // ------------------------------------------------------- lifecycle -----
  void alloc_pdata(int cpu) override { E.parts[cpu]->priv = std::make_unique<SedfPcpu>(); }
  void free_pdata(int cpu) override {
    SedfPcpu& p = pc(cpu);
    for (auto* l : {&p.runq, &p.waitq})
      for (int sid : *l) sv(*E.slots[sid]).q = Q_NONE;
    for (int i : {PEN_Q, UTIL_Q})
      for (int sid : p.extraq[i]) sv(*E.slots[sid]).on_extra[i] = false;
    E.parts[cpu]->priv.reset();
  }
  int init_domain(Tenant& d) override {
    d.priv = std::make_unique<SedfDom>();
    return 0;
  }
  void destroy_domain(Tenant& d) override {
    d.priv.reset();
    adjust_weights();
  }
  void alloc_vdata(Slot& v) override { v.priv = std::make_unique<SedfSlot>(); }
  void insert_vcpu(Slot& v) override {
    if (v.is_idle()) return;
    if (Tenant* t = E.tenant(v.tenant); t && t->priv) apply(*t, v);
  }
  void remove_vcpu(Slot& v) override {
    del_from_queue(v);
    extraq_del(v, PEN_Q);
    extraq_del(v, UTIL_Q);
  }

  // ------------------------------------------------------ parameters -----
  void apply(Tenant& d, Slot& v) {
    SedfDom& p = sd(d);
    SedfSlot& s = sv(v);
    s.latency = p.latency * kUs;
    if (p.weight) {
      if (p.extratime && !p.period) {  // weight-driven, extra time only
        s.extraweight = p.weight;
        s.weight = 0;
        s.slice = s.slice_orig = 0;
        s.period = s.period_orig = kWeightPeriod;
      } else {  // weight-driven real-time: slice set by adjust_weights
        s.weight = p.weight;
        s.extraweight = 0;
      }
    } else {
      s.weight = 0;
      s.extraweight = p.extratime ? 1 : 0;
      s.period = s.period_orig = p.period * kUs;
      s.slice = s.slice_orig = p.slice * kUs;
    }
    if (p.extratime)
      s.status |= EXTRA_AWARE;
    else {
      s.status &= ~EXTRA_AWARE;
      extraq_del(v, UTIL_Q);
    }
  }

  // sedf_adjust_weights: per partition, weight-driven slots share what the
  // time-driven reservations leave of WEIGHT_PERIOD (minus WEIGHT_SAFETY).
  void adjust_weights() {
    std::vector<int64_t> sumw(E.parts.size(), 0), sumt(E.parts.size(), 0);
    for (auto& tp : E.tenants) {
      if (!tp || !tp->alive || tp->pool != pool_ || !tp->priv) continue;
      for (int sid : tp->slots) {
        SedfSlot& s = sv(*E.slots[sid]);
        const int c = E.slots[sid]->processor;
        if (s.weight)
          sumw[c] += s.weight;
        else if (s.period_orig > 0)
          sumt[c] += kWeightPeriod * s.slice_orig / s.period_orig;
      }
    }
    for (auto& tp : E.tenants) {
      if (!tp || !tp->alive || tp->pool != pool_ || !tp->priv) continue;
      for (int sid : tp->slots) {
        SedfSlot& s = sv(*E.slots[sid]);
        const int c = E.slots[sid]->processor;
        if (!s.weight || !sumw[c]) continue;
        s.period = s.period_orig = kWeightPeriod;
        s.slice = s.slice_orig = std::max<int64_t>(0, s.weight * (kWeightPeriod - kWeightSafety - sumt[c]) / sumw[c]);
      }
    }
  }

  int adjust_ext(Tenant& d, bool set, gpbs_sched_ext_t& x) override {
    SedfDom& p = sd(d);
    if (set) {
      if (!x.period_us && !x.weight) return GPBS_EINVAL;
      if (x.weight) {
        p.weight = x.weight;
        if (x.extratime >= 0) p.extratime = x.extratime ? 1 : 0;
        if (p.extratime && !x.period_us) p.period = 0;
      } else {
        const int64_t per = (int64_t)x.period_us * kUs, sl = (int64_t)x.slice_us * kUs;
        if (per > kPeriodMax || per < kPeriodMin || sl > per || sl < kSliceMin) return GPBS_EINVAL;
        p.weight = 0;
        p.period = x.period_us;
        p.slice = x.slice_us;
        if (x.extratime >= 0) p.extratime = x.extratime ? 1 : 0;
      }
      if (x.latency_us >= 0) p.latency = x.latency_us;
      for (int sid : d.slots) apply(d, *E.slots[sid]);
      adjust_weights();
      for (int sid : d.slots) {  // re-evaluate now
        Slot& v = *E.slots[sid];
        E.raise_softirq(v.processor);
      }
    }
    const SedfSlot* s0 = d.slots.empty() ? nullptr : &sv(*E.slots[d.slots[0]]);
    x.period_us = s0 ? (int32_t)(s0->period_orig / kUs) : (int32_t)p.period;
    x.slice_us = s0 ? (int32_t)(s0->slice_orig / kUs) : (int32_t)p.slice;
    x.latency_us = (int32_t)p.latency;
    x.extratime = p.extratime;
    x.weight = p.weight;
    x.credit = s0 ? (int32_t)((s0->slice - s0->cputime) / kUs) : 0;
    return GPBS_OK;
  }

  int adjust(Tenant& d, bool set, int* weight, int* cap) override {
    // Generic weight/cap: weight drives sedf's weight mode (extra time kept).
    if (set && *weight != -1 && *weight != 0) {
      if (*weight < 1 || *weight > GPBS_WEIGHT_MAX) return GPBS_ERANGE;
      gpbs_sched_ext_t x{};
      x.weight = *weight;
      x.extratime = -1;
      x.latency_us = -1;
      int rc = adjust_ext(d, true, x);
      if (rc) return rc;
    }
    *weight = sd(d).weight;
    *cap = 0;
    return GPBS_OK;
  }
  int adjust_global(bool set, int* tslice_us, int* ratelimit_us) override {
    if (set) return GPBS_EINVAL;
    *tslice_us = (int)(kExtraQuantum / kUs);
    *ratelimit_us = 0;
    return GPBS_OK;
  }

  // ---------------------------------------------------- observability ----
  uint32_t trace_word(Slot& v) override {
    if (!v.priv || v.is_idle()) return 0;
    const int64_t left = std::clamp<int64_t>((sv(v).slice - sv(v).cputime) / kUs, -(1 << 23), (1 << 23) - 1);
    return (uint32_t)(128 + (extra_runs(sv(v)) ? -1 : 0)) | ((uint32_t)left << 8);
  }
  void fill_tenant_info(Tenant& d, gpbs_tenant_info_t& o) override {
    SedfDom& p = sd(d);
    o.weight = p.weight;
    o.cap = 0;
    const SedfSlot* s0 = d.slots.empty() ? nullptr : &sv(*E.slots[d.slots[0]]);
    o.tslice_us = s0 ? (uint32_t)(s0->slice_orig / kUs) : 0;
    o.tick_period_us = s0 ? (uint32_t)(s0->period_orig / kUs) : 0;
  }
  void fill_slot_info(Slot& v, gpbs_slot_info_t& o) override {
    SedfSlot& s = sv(v);
    o.credit = (int32_t)std::clamp<int64_t>((s.slice - s.cputime) / kUs, INT32_MIN, INT32_MAX);
    o.on_runq = s.q != Q_NONE;
    o.pri = s.q == Q_RUN ? 1 : (s.on_extra[PEN_Q] || s.on_extra[UTIL_Q] ? 0 : -1);
  }
  void dump_settings(std::string& o) override { o += efmt("Scheduler: %s (%s)\n", name(), opt_name()); }
  void dump_slot(Slot& v, std::string& o) {
    SedfSlot& s = sv(v);
    o += efmt("%i.%i has=%c p=%lld sl=%lld ddl=%lld w=%i c=%lld sc=%i xtr(%s)=%lld ew=%hu", v.tenant, v.index,
              v.is_running ? 'T' : 'F', (long long)(s.period / kUs), (long long)(s.slice / kUs),
              (long long)(s.deadl_abs / kUs), s.weight, (long long)(s.cputime / kUs), (int)s.score[UTIL_Q],
              (s.status & EXTRA_AWARE) ? "yes" : "no", (long long)(s.extra_time_tot / kUs),
              (unsigned short)s.extraweight);
    if (s.block_tot)
      o += efmt(" sb=%llu lb=%llu", (unsigned long long)s.short_block_tot, (unsigned long long)s.long_block_tot);
    o += "\n";
  }
  void dump_cpu_state(int cpu, std::string& o) override {
    SedfPcpu& p = pc(cpu);
    o += efmt("now=%lld\n", (long long)(E.now() / kUs));
    const char* names[4] = {"RUNQ", "WAITQ", "EXTRAQ (penalty)", "EXTRAQ (utilization)"};
    const std::list<int>* ls[4] = {&p.runq, &p.waitq, &p.extraq[PEN_Q], &p.extraq[UTIL_Q]};
    for (int k = 0; k < 4; ++k) {
      o += efmt("%s rq %p   n: %zu\n", names[k], (const void*)ls[k], ls[k]->size());
      int n = 0;
      for (int sid : *ls[k]) {
        o += efmt("  %3d: ", n++);
        dump_slot(*E.slots[sid], o);
      }
    }
  }
  void dump_admin_conf(std::string& o) override {
    for (auto& tp : E.tenants) {
      if (!tp || !tp->alive || tp->pool != pool_ || !tp->priv) continue;
      SedfDom& p = sd(*tp);
      o += efmt("dom%d period=%lldus slice=%lldus latency=%lldus extra=%d weight=%d missed=", tp->id,
                (long long)p.period, (long long)p.slice, (long long)p.latency, p.extratime, p.weight);
      uint64_t m = 0;
      for (int sid : tp->slots) m += sv(*E.slots[sid]).missed;
      o += efmt("%llu\n", (unsigned long long)m);
    }
  }
  std::string check() override {
    for (auto& tp : E.tenants) {
      if (!tp || !tp->alive || tp->pool != pool_ || !tp->priv) continue;
      for (int sid : tp->slots) {
        Slot& v = *E.slots[sid];
        SedfSlot& s = sv(v);
        if (s.q == Q_RUN && !has_pc(v.processor)) return efmt("sedf: slot %d queued on a partition outside the pool", sid);
        if ((s.on_extra[PEN_Q] || s.on_extra[UTIL_Q]) && (s.status & SEDF_ASLEEP) && !v.is_running)
          return efmt("sedf: sleeping slot %d on an extra queue", sid);
      }
    }
    return "";
  }
};

}  // namespace

std::unique_ptr<Scheduler> make_sedf_scheduler(Engine& e, int pool) {
  return std::make_unique<SedfScheduler>(e, pool);
}

}  // namespace gpbs
