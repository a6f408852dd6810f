/* libgpbs — stable C ABI of the gpbs co-scheduler (the libxl/libxc analog).
 *
 * Terminology map:  domain -> tenant, vCPU -> slot,
 * pCPU -> partition (an XCD-aligned CU group of one GPU), cpupool -> pool.
 *
 * Reference control surface: X:tools/libxl/libxl.c:3987-4116 (sched params),
 * X:xen/include/public/sysctl.h:568-579 (tslice/ratelimit ABI),
 * X:xen/include/public/domctl.h:309-329 (weight/cap).
 */
#ifndef GPBS_H
#define GPBS_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPBS_ABI_VERSION 6

/* Validation ranges (sysctl.h:568-579, libxl.c:4026-4101). Q1: the new API
 * also accepts the reference's boot default of 100us (see docs). */
#define GPBS_TSLICE_UMIN 100
#define GPBS_TSLICE_UMAX 1000000
#define GPBS_TSLICE_XL_UMIN 1000
#define GPBS_RATELIMIT_MIN 100
#define GPBS_RATELIMIT_MAX 500000
#define GPBS_WEIGHT_DEFAULT 256
#define GPBS_WEIGHT_MAX 65535

/* Error codes (negative errno style, mirrored in pbs_amd/core/errors.py). */
#define GPBS_OK 0
#define GPBS_EINVAL -22
#define GPBS_ENOENT -2
#define GPBS_EBUSY -16
#define GPBS_ENOMEM -12
#define GPBS_ERANGE -34
#define GPBS_ENOSPC -28
#define GPBS_EEXIST -17
#define GPBS_EIO -5

typedef struct gpbs_adapt_params {
  uint32_t threshold, band_lo, band_hi, min_us, max_us, inc_us, dec_us, switch_boundary;
  uint32_t ticks_per_tslice, spin_floor, scale, strict_ref;
  uint32_t grow_pct; /* 0: the reference's additive steps; >0: proportional growth (adapt_impl.h) */
} gpbs_adapt_params_t;

typedef struct gpbs_atc_params {
  uint32_t default_us, min_us, max_us, zero_step_us, climb_step_us, climb_floor_us, base_us, slope_us,
      alpha, warmup, apply_period_us,
      wait_unit_ns; /* reported wait ns per reference spin iteration (0/1 = raw) */
} gpbs_atc_params_t;

/* Boot parameters (level-1 config; X:xen/common/schedule.c:39-54,
 * X:xen/common/sched_credit.c:124-127,545,728). */
typedef struct gpbs_boot_params {
  char sched[16];              /* "credit" (PBS adaptive credit, default), "credit-fixed", "atc", "static" */
  int32_t tslice_us;           /* sched_credit_tslice_us, default 100 */
  int32_t ratelimit_us;        /* sched_ratelimit_us, default 1000 (clamped to tslice) */
  int32_t smt_power_savings;   /* sched_smt_power_savings */
  int32_t tickle_one_idle;     /* tickle_one_idle_cpu, default 1 */
  int32_t default_yield;       /* sched_credit_default_yield */
  int32_t migration_delay_us;  /* vcpu_migration_delay */
  int32_t metric_period_us;    /* CSCHED_METRIC_TICK_PERIOD, default 1000 */
  int32_t slice_apply_us;      /* CSCHED_TIME_APPLY, default 3000 */
  int32_t sim_clock;           /* 1 = deterministic simulated clock (tests / replay) */
  int32_t pmu_refresh_us;      /* 1111: tick-vs-metric PMU refresh split (sched_credit.c:456,1538) */
  int32_t dom0_quirk;          /* 1 = reference credit ceiling for tenant 0 (P1g) */
  int32_t heartbeat_timeout_us;/* 0 = off; tenants missing heartbeats are reaped */
  int32_t trace_capacity;      /* trace ring records (power of two), default 65536 */
  int32_t quantum_align_us;    /* 0 = off; round quantum expiries up to this grid (batched switches) */
  int32_t coschedule;          /* 1 = contention-aware sibling selection; 2 = + counter-driven context classes */
  int32_t class_period_us;     /* contention-class re-evaluation period, default 2000 */
  int32_t boost_exclusive;     /* 1 = memory-class slots park while a sibling context of their XCD runs a BOOSTed waker */
  int32_t class_split;         /* contexts [0, class_split) of an XCD host the compute class, the rest the memory class;
                                  0/1 = context 0 only.  > 1 also makes each class one gang (SE-exclusive mode) */
  int32_t idle_skip;           /* 1 = PBS idle-sample rule (Q14): a tenant with no counted instructions in a metric
                                  period is not fed to the phase detector (curr = 0 would shrink its quantum) */
  int32_t class_dwell;         /* class re-evaluations a new contention class must persist before a tenant is
                                  re-homed (default 2); the classifier also has a +-25 % band around the threshold */
  int32_t class_budget;        /* 1 = demand-driven SE budgets (class_split > 1): each PRESENT classified tenant gets a
                                  set of shader engines sized by the classes present (aligned halves, singles, or the
                                  class region time-shared when it has more tenants than SEs); surplus slots go offline
                                  (vcpu-set) -- no bench-side slot counts decide the layout.  2 = the same, but a
                                  crowded region is split by blocks of whole XCDs instead of time-shared */
  int32_t present_us;          /* class_budget: a tenant with no runnable slot for this long leaves the layout
                                  (default 10000) */
  int32_t sibling_steal;       /* class_budget: 1 = let an in-class steal stack a tenant's slot onto a partition that
                                  already holds a runnable sibling (Xen semantics); 0 (default) skips such a peer slot --
                                  in a time-shared region every tenant has a home on every partition, so the steal is
                                  zero-sum and the class tick undoes it */
  int32_t class_steal;         /* class_budget: 1 (default) = an idle partition may steal a slot of the other class
                                  (Xen 4.5's second balance step, work conservation); 0 = only the relayout after
                                  present_us hands an absent class's partitions over -- a short gap in one tenant's
                                  work no longer pulls the other class's runner onto an unmasked queue */
  int32_t class_fall;          /* contention classes: the smoothed miss rate follows a DROP at alpha 1/2 instead of
                                  1/4 (a rise already crosses the threshold in one sample): a memory-bound phase
                                  that ends is re-classified in ~6 periods instead of ~14.  0 = symmetric 1/4 */
  int32_t shared_q_us;         /* class_budget: a time-shared class region rotates at least this quantum (PBS mode;
                                  0 = the largest adaptive quantum of its co-sharers only) */
  int32_t class_pin_us;        /* class_budget: a tenant whose last THREE class changes fall within this window is
                                  laid out as memory class (its region time-shares; it takes no compute SEs from a
                                  compute tenant) until it settles.  0 = off */
  int32_t region_q;            /* class_budget, time-shared class region: 0 = every tenant runs its OWN quantum (PBS:
                                  its adaptive quantum, at least its switch-cost floor); 1 = the round-5 region quantum
                                  (the largest adaptive quantum of the co-sharers, floored at shared_q_us) */
  int32_t switch_floor_x;      /* per-tenant quantum floor in a time-shared region = this x the tenant's measured
                                  switch cost (revocation drain + re-entry ramp, gpbs_tenant_switch_cost); 0 = off */
  int32_t switch_floor_max_us; /* ... capped here (0 = max_us) */
  int32_t region_vt;           /* 1 = a time-shared region picks its next tenant by least region virtual time (owned
                                  partition-time / weight) among the runnable co-sharers, BOOSTed wakers first, so
                                  per-tenant quanta of any length stay weight-fair; 0 = credit priority + runq order */
  int32_t slo_cap;             /* 1 = a co-sharer's quantum in a region that holds a tenant with a latency target
                                  (gpbs_tenant_slo) is capped so the target's waiting time fits the target */
  int32_t probe_max_us;        /* class_budget: a present tenant still unclassified after this long (its tenures are
                                  too short for a clean counter window: a latency tenant's 50 us requests) is laid out
                                  as memory class instead of holding every tenant in the probe layout; 0 = no limit */
  int32_t mem_split;           /* class_budget 1: a crowded MEMORY-class region is split among its tenants by
                                  partitions (blocks of (shader engine, XCD) in context-major order) instead of
                                  time-shared: each backlogged tenant an equal block, a light tenant (busy at under
                                  half of the class ticks: a latency tenant) a small one.  Memory-bound tenants are
                                  bandwidth-bound well below a whole region (concave in CUs), and tenants bound by
                                  different paths (HBM vs the MALL) overlap; a crowded compute region stays
                                  time-shared (a GEMM needs its tile count of CUs).  2 = the light tenants' blocks
                                  overlap the last backlogged tenant's (a request BOOST-preempts it there) instead of
                                  idling between requests.  0 = time-share */
  gpbs_adapt_params_t adapt;
  gpbs_atc_params_t atc;
} gpbs_boot_params_t;

typedef struct gpbs_engine gpbs_engine_t;

/* Per-tenant adaptation state (device/host shared layout, see adapt.h). */
typedef struct gpbs_filter_entry { uint64_t spin, inst, miss; } gpbs_filter_entry_t;
typedef struct gpbs_adapt_state {
  uint32_t tslice_us, tick_period_us, window_left, stable_count, phase;
  int32_t last_err;
  int64_t last_curr, last_win;
  gpbs_filter_entry_t filter[5];
} gpbs_adapt_state_t;

/* Counter backend (vPMU analog).  All callbacks run under the engine lock. */
typedef struct gpbs_counter_ops {
  void* user;
  /* pmu_save_regs analog: refresh cumulative pmc[4] of a slot. may be NULL */
  int (*slot_refresh)(void* user, int slot_id, int tenant, int partition, uint64_t* pmc);
  /* Tenant-delta mode: deltas since the previous call for n tenants (out[4*n]).
   * When non-NULL it replaces the per-slot pmc reduction. */
  int (*tenant_deltas)(void* user, int n, const int* tenants, uint64_t* out);
  /* Optional batched adaptation (device kernel).  Updates states in place. */
  int (*adapt_batch)(void* user, int n, const int* tenants, const uint64_t* deltas, const uint64_t* spin_sum,
                     const uint64_t* spin_cnt, gpbs_adapt_state_t* states, const gpbs_adapt_params_t* p);
  /* Asynchronous device adaptation (preferred over adapt_batch when both are
   * set; the metric tick never waits on the GPU): adapt_launch starts this
   * period's PBS update of n tenants (0, or < 0 when it cannot start now --
   * the tick then adapts on the host); adapt_harvest returns the previous
   * launch's results once complete (count, tenants_out / states_out) or -11
   * while it still runs.  tenants_out is in/out: on entry it holds the
   * caller's launched tenant ids (max of them), and only a launch of exactly
   * those tenants is harvested -- several pools may share one backend, each
   * harvests its own launch (-22 if there is none).  The engine applies
   * results one metric period late and recomputes a late period on the host
   * (bit-identical). */
  int (*adapt_launch)(void* user, int n, const int* tenants, const uint64_t* deltas, const uint64_t* spin_sum,
                      const uint64_t* spin_cnt, const gpbs_adapt_state_t* states, const gpbs_adapt_params_t* p);
  int (*adapt_harvest)(void* user, int max, int* tenants_out, gpbs_adapt_state_t* states_out);
} gpbs_counter_ops_t;

/* Actuator (context switch analog).  on_switch is called for every partition
 * switch; on_flush once after each batch of engine work (one device-side
 * partition table update per batch). */
typedef struct gpbs_actuator_ops {
  void* user;
  void (*on_switch)(void* user, int partition, int prev_tenant, int next_tenant, int next_slot, int32_t quantum_us,
                    int64_t now_ns);
  void (*on_flush)(void* user, int64_t now_ns);
  void (*on_park)(void* user, int tenant, int slot, int parked);
} gpbs_actuator_ops_t;

/* Trace record (32 B), see csrc/obs/trace.h for event codes. */
/* Per-GPU backend multiplexer: an engine spanning several GPUs drives one
 * actuator + counter backend per GPU.  Backend i serves partitions
 * [part_lo, part_hi) (disjoint ranges): switch events go to the backend whose
 * range holds the partition, flushes and parks to all, and tenant counter
 * deltas are summed over the backends.  Installs the mux as the engine's
 * actuator/counter ops; returns the backend index or an error. */
int gpbs_backend_mux_add(struct gpbs_engine* e, int part_lo, int part_hi, const gpbs_actuator_ops_t* act,
                         const struct gpbs_counter_ops* ctr);
int gpbs_backend_mux_clear(struct gpbs_engine* e);
int gpbs_backend_mux_count(struct gpbs_engine* e);

/* Fault-injection point outside the engine (gang thread, control-page
 * writer): returns the kind's param (>= 0) when it fires, -1 otherwise. */
int64_t gpbs_fault_fire(struct gpbs_engine* e, const char* kind);
/* The gang epoch missed its deadline on this rank: clear every cross-GPU gang
 * window, count it (perfc gang_timeout) and trace GANG_TIMEOUT. */
int gpbs_gang_timeout(struct gpbs_engine* e, uint32_t epoch, uint32_t rank, uint32_t waited_us);

typedef struct gpbs_trace_record {
  uint64_t t_ns;
  uint32_t event, cpu;
  uint32_t a[4];
} gpbs_trace_record_t;

typedef struct gpbs_tenant_info {
  int32_t id, pool, nslots, weight, cap, paused, alive, active_slots;
  uint32_t tslice_us, tick_period_us, phase, window_left;
  int32_t last_err;
  int32_t shutdown;         /* 0, or GPBS_SHUTDOWN_WATCHDOG */
  int64_t last_curr, last_win;
  uint64_t pmc[4];          /* last per-tenant deltas (INST, CYC, REF, MISS) */
  uint64_t cache_miss_rate, cpi; /* per 100k inst, per 1k inst */
  uint64_t spin_latency, report_count, pending_requests, sched_count;
  int64_t run_ns;           /* total running time across slots */
  char name[64];
  int32_t online_slots;     /* slots not offline (vcpu-set / class_budget) */
  uint32_t budget_ctx;      /* class_budget: contexts (shader engines) of every XCD the layout gave it (bit c) */
  int32_t budget_shared;    /* class_budget: its class region is time-shared */
  uint32_t target_tslice_us;/* the policy's quantum target (PBS: the adaptive tslice); tslice_us above is the
                               quantum the dispatcher gives the tenant now (region floors / caps applied) */
  uint32_t switch_cost_us;  /* measured switch cost (drain + ramp, EWMA) the engine holds for the tenant */
  uint32_t slo_us;          /* latency target, 0 = none */
  uint32_t last_dispatch_us;/* the quantum of its last dispatch (0: never dispatched) */
} gpbs_tenant_info_t;

typedef struct gpbs_slot_info {
  int32_t id, tenant, index, processor, pri, flags, runstate, is_running, credit, on_runq;
  uint64_t pmc[4];
  uint64_t sched_count;
  int64_t run_ns, runnable_ns, blocked_ns;
  uint64_t affinity[4];
  int32_t class_home;   /* contention-class / budget home partition, -1 none */
  uint32_t pause_flags; /* VPF_* (1 blocked, 2 migrating, 4 offline) */
} gpbs_slot_info_t;

/* Scheduler-specific per-tenant parameters (xl sched-credit2 / sched-sedf).
 * credit2: weight.  sedf: period/slice/latency (us), extratime (0/1), weight
 * (weight-driven reservation; 0 = time-driven).  -1 = leave unchanged where
 * noted.  credit (out): credit2 credit / sedf remaining slice, us. */
typedef struct gpbs_sched_ext {
  int32_t weight, period_us, slice_us, latency_us, extratime, credit;
} gpbs_sched_ext_t;

typedef struct gpbs_partition_info {
  int32_t id, gpu, xcd, pool, curr_tenant, curr_slot, runq_len, idle, ctx, reserved;
  uint64_t switches;
} gpbs_partition_info_t;

/* ARINC 653 schedule (xen_sysctl_arinc653_schedule, public/sysctl.h:545-566):
 * a major frame of windows, each owned by a tenant (slot -1: all of its
 * slots; slot k: that slot only).  Times in ns. */
#define GPBS_ARINC653_MAX_ENTRIES 64
typedef struct gpbs_arinc653_entry {
  int32_t tenant, slot;
  int64_t runtime_ns;
} gpbs_arinc653_entry_t;
typedef struct gpbs_arinc653_schedule {
  int64_t major_frame_ns;
  int32_t num_entries, is_explicit; /* get: 0 = the automatic table */
  gpbs_arinc653_entry_t entries[GPBS_ARINC653_MAX_ENTRIES];
} gpbs_arinc653_schedule_t;
/* put / get the pool's table; GPBS_EINVAL if the pool is not arinc653 or the
 * table is invalid (frame <= 0, no entries, runtime <= 0, sum > frame). */
int gpbs_arinc653_set(gpbs_engine_t* e, int pool, const gpbs_arinc653_schedule_t* s);
int gpbs_arinc653_get(gpbs_engine_t* e, int pool, gpbs_arinc653_schedule_t* s);

/* --- scheduler-specific tenant parameters (S4: credit2, sedf) --- */
int gpbs_sched_ext(gpbs_engine_t* e, int tenant, int set, gpbs_sched_ext_t* p);
/* ATC pool across GPUs: applies global_min_us (> 0) and returns the pool's
 * local minimum slice of its last apply (us); GPBS_EINVAL if not ATC. */
int gpbs_atc_sync(gpbs_engine_t* e, int pool, int global_min_us);

/* --- lifecycle --- */
void gpbs_boot_defaults(gpbs_boot_params_t* p);
gpbs_engine_t* gpbs_engine_create(const gpbs_boot_params_t* p);
void gpbs_engine_destroy(gpbs_engine_t* e);
int gpbs_abi_version(void);
const char* gpbs_strerror(int err);

/* --- topology / pools (cpupool analog, X:xen/common/cpupool.c) --- */
int gpbs_partition_add(gpbs_engine_t* e, int gpu, int xcd);       /* -> partition id, free (no pool) */
int gpbs_partition_add_ctx(gpbs_engine_t* e, int gpu, int xcd, int ctx); /* XCD issue context (sibling) */
int gpbs_pool_create(gpbs_engine_t* e, const char* name, const char* sched); /* -> pool id */
int gpbs_pool_destroy(gpbs_engine_t* e, int pool);
int gpbs_pool_rename(gpbs_engine_t* e, int pool, const char* name);
int gpbs_pool_find(gpbs_engine_t* e, const char* name);
int gpbs_pool_assign(gpbs_engine_t* e, int pool, int partition);   /* cpupool-cpu-add */
int gpbs_pool_unassign(gpbs_engine_t* e, int pool, int partition); /* cpupool-cpu-remove */
int gpbs_pool_info(gpbs_engine_t* e, int pool, char* name, int name_len, char* sched, int sched_len,
                   uint64_t* mask4, int* n_tenants);
int gpbs_pool_list(gpbs_engine_t* e, int* ids, int max);
int gpbs_partition_info(gpbs_engine_t* e, int partition, gpbs_partition_info_t* out);
int gpbs_num_partitions(gpbs_engine_t* e);

/* --- tenants / slots (domain/vcpu analog) --- */
int gpbs_tenant_create(gpbs_engine_t* e, const char* name, int pool, int nslots, int weight, int cap);
int gpbs_tenant_destroy(gpbs_engine_t* e, int tenant);
int gpbs_tenant_find(gpbs_engine_t* e, const char* name);
int gpbs_tenant_list(gpbs_engine_t* e, int* ids, int max);
int gpbs_tenant_move(gpbs_engine_t* e, int tenant, int pool);      /* cpupool-migrate */
int gpbs_tenant_pause(gpbs_engine_t* e, int tenant);
int gpbs_tenant_unpause(gpbs_engine_t* e, int tenant);
int gpbs_tenant_set_nslots(gpbs_engine_t* e, int tenant, int nslots); /* vcpu-set: online count */
int gpbs_slot_id(gpbs_engine_t* e, int tenant, int index);
int gpbs_slot_wake(gpbs_engine_t* e, int tenant, int index);      /* index -1: all slots */
int gpbs_slot_block(gpbs_engine_t* e, int tenant, int index);     /* index -1: all slots */
int gpbs_slot_yield(gpbs_engine_t* e, int tenant, int index);
int gpbs_slot_pin(gpbs_engine_t* e, int tenant, int index, const uint64_t* mask4); /* vcpu-pin */
int gpbs_tenant_info(gpbs_engine_t* e, int tenant, gpbs_tenant_info_t* out);
int gpbs_tenant_class(gpbs_engine_t* e, int tenant); /* contention class: 0 compute, 1 memory, -1 unknown */
/* Metric periods with a measurement / with the quantum at min_us / at max_us
 * (credit modes); reset != 0 clears them after the read. */
int gpbs_tenant_bound_stats(gpbs_engine_t* e, int tenant, uint64_t* out3, int reset);
/* Measurement tenure: the tenant's next tenure (on any partition) lasts at
 * least `us` (0 cancels, UINT32_MAX only reads); returns the tenures so
 * extended so far, or <0. */
int gpbs_tenant_measure(gpbs_engine_t* e, int tenant, uint32_t us);
/* Measured cost of one switch of the tenant's partitions (revocation drain +
 * re-entry ramp, ns; the GPU runtime's EWMA): the per-tenant quantum floor of
 * a time-shared region (boot switch_floor_x).  0 clears it. */
int gpbs_tenant_switch_cost(gpbs_engine_t* e, int tenant, uint64_t ns);
/* Latency target of a tenant (us; 0 = none): with boot slo_cap, the quanta of
 * its co-sharers in a time-shared region are capped so it waits at most this
 * long for a turn. */
int gpbs_tenant_slo(gpbs_engine_t* e, int tenant, uint32_t us);
/* Cumulative INST, CYCLES, LLC refs, LLC misses the scheduler measured and
 * attributed to the tenant (sum over metric periods; the vPMU mirror). */
int gpbs_tenant_vpmu(gpbs_engine_t* e, int tenant, uint64_t* total4);
int gpbs_slot_info(gpbs_engine_t* e, int slot, gpbs_slot_info_t* out);
int gpbs_tenant_adapt_state(gpbs_engine_t* e, int tenant, gpbs_adapt_state_t* out, int set);
int gpbs_tenant_heartbeat(gpbs_engine_t* e, int tenant);

/* --- scheduler control (sched-credit) --- */
int gpbs_sched_credit_get(gpbs_engine_t* e, int tenant, int* weight, int* cap);
int gpbs_sched_credit_set(gpbs_engine_t* e, int tenant, int weight, int cap); /* -1 = leave */
int gpbs_sched_params_get(gpbs_engine_t* e, int pool, int* tslice_us, int* ratelimit_us);
int gpbs_sched_params_set(gpbs_engine_t* e, int pool, int tslice_us, int ratelimit_us);
int gpbs_sched_name(gpbs_engine_t* e, int pool, char* out, int len);

/* --- paravirtual report channel (vcrd_op analog, P2) --- */
int gpbs_report_wait(gpbs_engine_t* e, int tenant, uint64_t wait_ns, int kind);
int gpbs_report_requests(gpbs_engine_t* e, int tenant, uint64_t n); /* pending_requests (P7) */

/* --- host-CPU backend (config #1): perf_event counters + SIGSTOP/affinity gate --- */
#define GPBS_PERF_HW 1 /* instructions, cycles, LLC refs, LLC misses */
#define GPBS_PERF_SW 2 /* task-clock x2, minor/major faults (no hardware PMU) */
void* gpbs_perf_open(int pid, int cpu);
int gpbs_perf_read(void* h, uint64_t* out4);
int gpbs_perf_mode(void* h);
void gpbs_perf_close(void* h);
int gpbs_perf_available(void);
void* gpbs_gate_create(const char* mode); /* "signal" (default) */
int gpbs_gate_mode(void* g);
int gpbs_gate_add_pid(void* g, int tenant, int pid);
int gpbs_gate_set(void* g, int tenant, int cpu, int on);
int gpbs_gate_stats(void* g, uint64_t* signals, uint64_t* pins);
void gpbs_gate_destroy(void* g);
void* gpbs_cpu_backend_create(gpbs_engine_t* e, void* gate);
int gpbs_cpu_backend_map(void* backend, int partition, int host_cpu);
int gpbs_cpu_backend_add(void* backend, int tenant, int pid);
void gpbs_cpu_backend_destroy(void* backend);

/* --- fault injection: spec "kind=ppm[:param],...,seed=N" (also env GPBS_FAULT
 *     at engine creation); kinds counter_drop counter_reset heartbeat_drop
 *     actuate_delay timer_jitter (param = us late) --- */
int gpbs_fault_set(gpbs_engine_t* e, const char* spec);
int gpbs_fault_hits(gpbs_engine_t* e, uint64_t* out, int n);

/* --- cross-GPU gang windows (pbs_amd/parallel/gang.py) --- */
int gpbs_gang_set(gpbs_engine_t* e, int tenant, int state, int64_t until_ns); /* 0 none 1 favour 2 exclude */

/* Native gang coordinator (csrc/comm/gang_coord.cpp): the per-rank epoch loop
 * on the shm transport as a C++ thread bound to the engine. */
#define GPBS_GANG_MAX_TENANTS 32
typedef struct gpbs_gang_cfg {
  int32_t rank, ntenants, nmetric, metric_every;
  int32_t tenants[GPBS_GANG_MAX_TENANTS];        /* gang tenants (windows) */
  int32_t metric_tenants[GPBS_GANG_MAX_TENANTS]; /* node-metric SUM tenants */
  int64_t epoch_ns, slack_ns, deadline_ns, start_ns, join_ns;
  double share;          /* fraction of the 8-epoch period given to gang windows */
  int32_t atc_pool;      /* -1: no ATC exchange */
  int32_t wait_driven;   /* windows only while the worst rank's K10 wait is high */
  double wait_on_frac;   /* wait EWMA >= frac * epoch turns a tenant's windows on */
  int32_t wait_hold_epochs, reform;
  void (*roctx_push)(const char*); /* optional marker ranges (libgpbs_hip) */
  void (*roctx_pop)(void);
} gpbs_gang_cfg_t;

typedef struct gpbs_gang_stats {
  int64_t epochs, sync_p50_ns, sync_p99_ns, sync_max_ns, skew_p50_ns, skew_max_ns;
  int64_t timeouts, degraded, reforms, members, atc_global_us, metric_syncs, gang_switches, error, finished;
} gpbs_gang_stats_t;

void* gpbs_gang_coord_start(gpbs_engine_t* e, void* shm, int world, int nvals, const gpbs_gang_cfg_t* cfg);
int gpbs_gang_coord_stop(void* c, int64_t timeout_ns);
int gpbs_gang_coord_running(void* c);
int gpbs_gang_coord_stats(void* c, gpbs_gang_stats_t* out);
int gpbs_gang_coord_tenant(void* c, int i, int64_t out[3]);
int gpbs_gang_coord_metrics(void* c, int i, int64_t last[4], int64_t totals[4]);
int gpbs_gang_coord_history(void* c, int64_t* epochs, int32_t* states, int max);
void gpbs_gang_coord_destroy(void* c);

/* --- counters / actuation backends --- */
int gpbs_set_counter_ops(gpbs_engine_t* e, const gpbs_counter_ops_t* ops);
int gpbs_set_actuator_ops(gpbs_engine_t* e, const gpbs_actuator_ops_t* ops);
int gpbs_slot_set_pmc(gpbs_engine_t* e, int slot, const uint64_t* pmc4); /* fake/replay source */
int gpbs_get_actuator_ops(gpbs_engine_t* e, gpbs_actuator_ops_t* out);
int gpbs_get_counter_ops(gpbs_engine_t* e, gpbs_counter_ops_t* out);

/* --- tenant control pages (csrc/ipc/ctlpage.cpp): POSIX shm, seqlock,
 *     SPSC wait-report ring, futex doorbell; bridge to an engine --- */
void* gpbs_ctl_create(const char* name, int ntenants);
void* gpbs_ctl_open(const char* name);
void gpbs_ctl_close(void* ctl, int unlink_region);
int gpbs_ctl_ntenants(void* ctl);
int gpbs_ctl_assign(void* ctl, int page, int tenant);
void gpbs_ctl_publish(void* ctl, int page, uint32_t gate, uint64_t mask, uint32_t quantum_us, int32_t prio,
                      int32_t tenant, uint32_t epoch);
int gpbs_ctl_read(void* ctl, int page, uint32_t* gate, uint64_t* mask, uint32_t* quantum_us, int32_t* prio,
                  int32_t* tenant, uint32_t* epoch);
/* wait-report kinds carried by gpbs_report_wait / gpbs_ctl_report */
#define GPBS_REPORT_WAIT 1     /* spin / wait latency (vcrd_op) */
#define GPBS_REPORT_HOLD 2     /* lock hold time (lockstat holdtime) */
#define GPBS_REPORT_REQUESTS 3 /* request arrivals; wait_ns = count */
int gpbs_ctl_read_mask(void* ctl, int page, uint64_t* mask2, uint32_t* epoch);
/* vPMU mirror (tenant side, seqlock read): cumulative counters the scheduler
 * attributed to the tenant, last period's miss rate (per 100k inst), current
 * quantum, contention class and PBS phase; *seq counts publications.  Returns
 * the retries (torn reads observed), or < 0. */
int gpbs_ctl_read_vpmu(void* ctl, int page, uint64_t* c4, uint64_t* miss_rate, uint32_t* tslice_us, int32_t* cls,
                       uint32_t* phase, uint32_t* seq);
int gpbs_ctl_report(void* ctl, int page, uint64_t wait_ns, uint32_t kind, uint32_t gpu);
int gpbs_ctl_drain(void* ctl, int page, uint64_t* waits, uint32_t* kinds, int max);
void gpbs_ctl_heartbeat(void* ctl, int page, uint64_t now_ns, uint32_t progress);
int gpbs_ctl_status(void* ctl, int page, uint64_t* heartbeat, uint64_t* dropped, uint32_t* has_work,
                    uint32_t* progress);
void gpbs_ctl_set_counters(void* ctl, int page, const uint64_t* c4);
void gpbs_ctl_get_counters(void* ctl, int page, uint64_t* c4);
void gpbs_ctl_set_work(void* ctl, int page, int has_work);
void gpbs_ctl_ring(void* ctl, int page);
int gpbs_ctl_doorbell_wait(void* ctl, int page, int64_t timeout_ns);
int gpbs_ctl_wait_gate(void* ctl, int page, int64_t timeout_ns);
int gpbs_ctl_bind(void* ctl, void* engine);

/* --- time --- */
int64_t gpbs_now(gpbs_engine_t* e);
int gpbs_advance(gpbs_engine_t* e, int64_t now_ns);  /* sim clock: run all events <= now */
int gpbs_start(gpbs_engine_t* e);                     /* real clock: start dispatcher thread */
int gpbs_stop(gpbs_engine_t* e);
int gpbs_poll(gpbs_engine_t* e);                      /* real clock: run due events once */
int64_t gpbs_next_event(gpbs_engine_t* e);

/* --- observability --- */
int gpbs_debug_keys(gpbs_engine_t* e, const char* keys, char* out, int len); /* r q z t ... */
int gpbs_dmesg(gpbs_engine_t* e, char* out, int len, int clear);
int gpbs_trace_read(gpbs_engine_t* e, uint64_t* cursor, gpbs_trace_record_t* out, int max, uint64_t* lost);
int gpbs_trace_set_mask(gpbs_engine_t* e, uint64_t mask);
int gpbs_trace_emit(gpbs_engine_t* e, uint32_t event, uint32_t cpu, uint32_t a0, uint32_t a1, uint32_t a2,
                    uint32_t a3);
int gpbs_perfc_count(void);
const char* gpbs_perfc_name(int i);
int gpbs_perfc_read(gpbs_engine_t* e, uint64_t* out, int max);
int gpbs_perfc_reset(gpbs_engine_t* e);
int gpbs_check_invariants(gpbs_engine_t* e, char* out, int len); /* CSCHED_VCPU_CHECK analog; 0 = ok */

/* Lock profile of the engine mutex (xenlockprof analog, X:xen/common/spinlock.c:88-115). */
typedef struct gpbs_lockprof {
  uint64_t lock_cnt, block_cnt, time_block_ns, time_hold_ns, max_block_ns, max_hold_ns, handoffs;
} gpbs_lockprof_t;
int gpbs_lockprof(gpbs_engine_t* e, gpbs_lockprof_t* out, int reset);

/* Tenant watchdogs (SCHEDOP_watchdog analog, X:xen/common/schedule.c:738-788):
 * id 0 allocates one of GPBS_WATCHDOGS timers and returns its id (1-based);
 * id > 0 re-arms it (timeout_ms > 0) or frees it (timeout_ms == 0).  A timer
 * that expires shuts the tenant down: its slots are paused and its info
 * reports shutdown = GPBS_SHUTDOWN_WATCHDOG. */
#define GPBS_WATCHDOGS 2
#define GPBS_SHUTDOWN_WATCHDOG 4
int gpbs_watchdog(gpbs_engine_t* e, int tenant, uint32_t id, uint32_t timeout_ms);

#ifdef __cplusplus
}
#endif
#endif /* GPBS_H */
