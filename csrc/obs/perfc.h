// Named performance counters (perfc analog: CSCHED_STAT_CRANK at
// X:xen/common/sched_credit.c:90, definitions X:xen/include/xen/perfc_defn.h:15-48,
// read by X:tools/misc/xenperf.c).  Names keep the csched:* vocabulary plus
// the PBS/gpbs additions listed in SURVEY §5.5.
#pragma once
#include <atomic>
#include <cstdint>

namespace gpbs {

#define GPBS_PERFC_LIST(X)                                                                            \
  X(sched_run) X(sched_ctx) X(schedule) X(acct_run) X(acct_no_work) X(acct_balance) X(acct_reorder)  \
  X(acct_min_credit) X(acct_vcpu_active) X(acct_vcpu_idle) X(vcpu_sleep) X(vcpu_wake_running)          \
  X(vcpu_wake_onrunq) X(vcpu_wake_runnable) X(vcpu_wake_not_runnable) X(vcpu_park) X(vcpu_unpark)     \
  X(tickle_local_idler) X(tickle_local_over) X(tickle_local_under) X(tickle_local_other)              \
  X(tickle_idlers_none) X(tickle_idlers_some) X(load_balance_idle) X(load_balance_over)               \
  X(load_balance_other) X(steal_trylock_failed) X(steal_peer_idle) X(migrate_queued)                  \
  X(migrate_running) X(dom_init) X(dom_destroy) X(vcpu_init) X(vcpu_destroy) X(vcpu_hot)              \
  X(vcpu_check) X(delay_ms) X(adapt_inc) X(adapt_dec) X(adapt_rearm) X(metric_tick) X(report_rx)     \
  X(gang_epoch) X(gang_timeout) X(counter_stale) X(counter_reset) X(tenant_dead) X(atc_apply) X(fault_injected)         \
  X(partition_switch) X(sched_irq) X(ratelimit_hold) X(boost_park) X(watchdog_fired) X(adapt_idle_skip) \
  X(class_change) X(relayout) X(adapt_device) X(adapt_late) X(probe_layout) X(probe_expired) X(wake_homed) X(mem_split) X(mirror) \
  X(steal_sibling_skip)

enum PerfcId : int {
#define GPBS_PERFC_ENUM(n) PC_##n,
  GPBS_PERFC_LIST(GPBS_PERFC_ENUM)
#undef GPBS_PERFC_ENUM
      PC_COUNT
};

extern const char* const kPerfcNames[PC_COUNT];

struct Perfc {
  std::atomic<uint64_t> v[PC_COUNT];
  Perfc() { reset(); }
  void incr(PerfcId id) { v[id].fetch_add(1, std::memory_order_relaxed); }
  uint64_t get(PerfcId id) const { return v[id].load(std::memory_order_relaxed); }
  void reset() {
    for (auto& x : v) x.store(0, std::memory_order_relaxed);
  }
};

}  // namespace gpbs
