// gpbs engine: the generic scheduling framework (analog of
// X:xen/common/schedule.c + cpupool.c + the vcpu/domain lifecycle in
// X:xen/common/domain.c), hosting pluggable policies behind Scheduler
// (X:xen/include/xen/sched-if.h:144-193).
//
// Design (MI355X-first): one engine per GPU-rank process.  Its partitions are
// XCD-aligned CU groups (8 per MI355X).  All partitions are driven by ONE
// dispatcher thread off a single timer heap (instead of per-pCPU softirqs);
// "IPIs" are softirq bits processed in the same pass.  External threads
// (tenant runners, the RPC server, the gang thread) enter through the C ABI
// under one engine mutex; wake-ups raise softirqs that are processed before
// the call returns, so a wake has µs latency without a context switch.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <vector>

#include "../include/gpbs/gpbs.h"
#include "../obs/lockprof.h"
#include "../obs/perfc.h"
#include "../obs/trace.h"
#include "adapt.h"
#include "bitmask.h"

namespace gpbs {

enum Pri : int16_t { PRI_BOOST = 0, PRI_UNDER = -1, PRI_OVER = -2, PRI_IDLE = -64 };
enum Runstate : int { RS_RUNNING = 0, RS_RUNNABLE = 1, RS_BLOCKED = 2, RS_OFFLINE = 3 };
constexpr uint32_t VPF_BLOCKED = 1u;    // _VPF_blocked
constexpr uint32_t VPF_MIGRATING = 2u;  // _VPF_migrating
constexpr uint32_t VPF_DOWN = 4u;       // _VPF_down (vcpu-set offline)

constexpr int kNumPmc = 4;  // INST, CYCLES, L2_REFS (LLC_REFERENCES), L2_MISSES (LLC_MISSES)

struct SchedSlotData {
  virtual ~SchedSlotData() = default;
};
struct SchedTenantData {
  virtual ~SchedTenantData() = default;
};
struct SchedPartData {
  virtual ~SchedPartData() = default;
};

struct Slot {  // struct vcpu
  int id = -1;
  int tenant = -1;  // -1: idle slot of a partition
  int index = 0;    // vcpu_id
  int processor = 0;
  int home = -1;        // one-shot placement hint for the next migration
  int class_home = -1;  // partition of this slot within its contention class
  int64_t homed_at = INT64_MIN / 2;  // last migration to class_home (steal guard)
  Mask affinity;        // hard affinity (vcpu-pin)
  Mask soft;            // soft affinity (contention class); empty = none
  uint32_t pause_flags = 0;
  int pause_count = 0;
  bool is_running = false;
  Runstate rs = RS_OFFLINE;
  int64_t rs_entry = 0;
  int64_t rs_time[4] = {0, 0, 0, 0};
  int64_t last_run_time = 0;
  uint64_t pmc[kNumPmc] = {0, 0, 0, 0};  // v->pmc (P4), cumulative
  uint64_t sched_count = 0;              // v->sched_count (P4)
  std::unique_ptr<SchedSlotData> priv;
  bool is_idle() const { return tenant < 0; }
};

struct Tenant {  // struct domain
  int id = -1;
  std::string name;
  int pool = 0;
  std::vector<int> slots;  // slot ids, index order
  int pause_count = 0;
  bool alive = true;
  bool pinned = false;
  uint64_t pending_requests = 0;  // P7 (live in gpbs: request-queue depth)
  int64_t last_heartbeat = 0;
  // Cumulative counters the scheduler measured/attributed for this tenant
  // (sum of the metric periods' deltas): what the vPMU mirror publishes on
  // its control page (Perfctr-xen's per-vCPU state page, S1/S2).
  uint64_t vpmu_total[4] = {0, 0, 0, 0};
  int cls = -1;          // contention class: 0 compute-bound (MFMA ctx), 1 memory-bound (memory ctx)
  // class_budget layout: last time any slot was runnable, and the contexts
  // (shader engines) the layout gave the tenant (bit c = ctx c), with the
  // XCDs in bits 8-15 when it is confined to a block of XCDs (0 = all; 0
  // overall = not placed / absent); budget_shared: its region is time-shared
  int64_t last_busy = INT64_MIN / 2;
  uint32_t budget_ctx = 0;
  bool budget_shared = false;
  int cls_pending = -1;  // hysteresis: a new class must be seen on consecutive ticks
  int cls_count = 0;
  int64_t cls_chg_ns[3] = {INT64_MIN / 2, INT64_MIN / 2, INT64_MIN / 2};  // last three confirmed class changes
  // class_pin_us: flapping = its last three class changes within the window
  bool flapping(int64_t now, int64_t pin_ns) const { return pin_ns > 0 && cls >= 0 && now - cls_chg_ns[0] <= pin_ns; }
  int lay_cls = -1;  // the class budget_layout placed it by (a pinned flapping tenant: 1)
  int64_t unclassified_since = INT64_MIN / 2;  // present and unclassified since (probe_max_us)
  bool probe_gaps = false;  // ... and seen blocked at a class tick meanwhile (short requests)
  // mem_split: share of class ticks the tenant was busy at (EWMA 1/16), and
  // whether the layout treats it as light (hysteresis 0.4 / 0.6)
  double busy_ewma = 1.0;
  bool light = false;
  // Cross-GPU gang window (parallel/gang.py): 1 favoured (run on every
  // partition that holds a slot), 2 excluded (its peers on other GPUs are not
  // running it), until gang_until (engine clock).
  int gang_state = 0;
  int64_t gang_until = 0;
  int gang(int64_t now) const { return now < gang_until ? gang_state : 0; }
  // Measurement tenure: the hardware-counter sampler asks that the tenant's
  // next tenure on some partition last at least measure_us, so a clean
  // counter window fits in it (a 1 ms quantum minus the drain guard and the
  // closing sample leaves none); granted = tenures so extended.
  uint32_t measure_us = 0;
  uint64_t measure_granted = 0;
  // Measured cost of one switch of its partitions (revocation drain + re-entry
  // ramp, the GPU runtime's EWMA; 0 = unknown) and its latency target (0 =
  // none): the per-tenant quantum floor / the co-sharers' cap in a
  // time-shared class region (credit.cpp pbs_quantum_us).
  uint32_t sw_cost_us = 0;
  uint32_t slo_us = 0;
  // Watchdogs (SCHEDOP_watchdog): timer ids, in-use bits, shutdown reason.
  int wd_timer[GPBS_WATCHDOGS] = {-1, -1};
  uint32_t wd_inuse = 0;
  int shutdown = 0;
  std::unique_ptr<SchedTenantData> priv;
};

struct Partition {  // pCPU + schedule_data
  int id = -1;
  int gpu = 0;
  int xcd = 0;
  int ctx = 0;  // issue context within the XCD (SMT-sibling analog)
  int pool = -1;
  int curr = -1;       // running slot (idle slot when idle)
  int idle_slot = -1;  // this partition's idle vCPU
  int s_timer = -1;
  bool softirq = false;
  uint64_t switches = 0;
  std::unique_ptr<SchedPartData> priv;
};

struct TaskSlice {
  int slot;
  int64_t time_ns;  // < 0: no limit
  bool migrated;
};

class Engine;

// One window of an ARINC 653 major frame (xen_sysctl_arinc653_schedule's
// sched_entries[]): the tenant (slot -1 = all its slots) and its runtime.
struct ArincEntry {
  int tenant;
  int slot;
  int64_t runtime;  // ns
};

// The pluggable scheduler interface (struct scheduler, sched-if.h:144-193).
class Scheduler {
 public:
  Scheduler(Engine& e, int pool) : E(e), pool_(pool) {}
  virtual ~Scheduler() = default;
  virtual const char* name() const = 0;
  virtual const char* opt_name() const = 0;
  virtual int init() { return 0; }
  virtual void deinit() {}
  virtual void alloc_pdata(int part) = 0;
  virtual void free_pdata(int part) = 0;
  virtual int init_domain(Tenant& d) = 0;
  virtual void destroy_domain(Tenant& d) = 0;
  virtual void alloc_vdata(Slot& v) = 0;
  virtual void insert_vcpu(Slot& v) = 0;
  virtual void remove_vcpu(Slot& v) = 0;
  virtual void sleep(Slot& v) = 0;
  virtual void wake(Slot& v) = 0;
  virtual void yield(Slot& v) = 0;
  virtual TaskSlice do_schedule(int part, int64_t now) = 0;
  virtual int pick_cpu(Slot& v) = 0;
  virtual int adjust(Tenant& d, bool set, int* weight, int* cap) = 0;
  virtual int adjust_global(bool set, int* tslice_us, int* ratelimit_us) = 0;
  // Scheduler-specific tenant parameters (credit2 weight, sedf reservation).
  virtual int adjust_ext(Tenant&, bool, gpbs_sched_ext_t&) { return GPBS_EINVAL; }
  // ATC across GPUs: local minimum slice out, node-wide minimum in (us).
  virtual int atc_sync(int) { return GPBS_EINVAL; }
  // ARINC 653 schedule table (a653sched_adjust_global put/get); get returns
  // 1 for an installed table, 0 for the automatic one.
  virtual int set_schedule(int64_t, const std::vector<ArincEntry>&) { return GPBS_EINVAL; }
  virtual int get_schedule(int64_t*, std::vector<ArincEntry>*) { return GPBS_EINVAL; }
  virtual void dump_settings(std::string& out) = 0;
  virtual void dump_cpu_state(int part, std::string& out) = 0;
  virtual void dump_admin_conf(std::string& out) = 0;
  virtual void tick_suspend(int) {}
  virtual void tick_resume(int) {}
  virtual void context_saved(Slot&) {}
  // gpbs additions: the paravirtual wait report routed by tenant id (Q6 fix)
  virtual void report(Tenant&, uint64_t, int) {}
  virtual bool tenant_adapt(Tenant&, AdaptState*) { return false; }
  // Metric periods with a measurement, and of those the ones whose quantum
  // sat at the adapt bounds (min_us, max_us); reset clears them.
  virtual int bound_stats(Tenant&, uint64_t*, bool) { return GPBS_EINVAL; }
  // Contention class from the counters: -1 unknown (no recent samples), 0 compute-bound, 1 memory-bound.
  virtual int classify(Tenant&) { return -1; }
  // A confirmed class change (after class_dwell): from -> to.
  virtual void class_changed(Tenant&, int, int) {}
  // Trace word of a slot: (priority + 128) in bits 0-7, credit (clamped to
  // +-2^23) in bits 8-31.  Carried by WAKE records (who could preempt whom).
  virtual uint32_t trace_word(Slot&) { return 0; }
  virtual bool set_tenant_adapt(Tenant&, const AdaptState&) { return false; }
  virtual void fill_tenant_info(Tenant&, gpbs_tenant_info_t&) {}
  virtual void fill_slot_info(Slot&, gpbs_slot_info_t&) {}
  virtual std::string check() { return ""; }
  int pool() const { return pool_; }

 protected:
  Engine& E;
  int pool_;
};

struct Pool {
  int id = -1;
  std::string name;
  std::string sched_name;
  Mask cpus;
  std::unique_ptr<Scheduler> sched;
  // contention classes present among the pool's classified tenants (bit c =
  // class c): the class layout the slots were last placed for (-1: none yet)
  int class_layout = -1;
  // class_budget: (tenant id, class) of the present tenants the budgets were
  // last computed for
  std::vector<std::pair<int, int>> budget_sig;
  std::vector<int> budget_light;  // mem_split: the light tenants of that layout
  // symmetric class halves (class_split = nctx / 2): the compute class holds
  // the upper half and the memory class the lower one (a mirrored layout)
  bool mirror = false;
};

std::unique_ptr<Scheduler> make_scheduler(const std::string& name, Engine& e, int pool);

class Engine {
 public:
  explicit Engine(const gpbs_boot_params_t& p);
  ~Engine();

  gpbs_boot_params_t boot;
  AdaptParams adapt_params;
  AtcParams atc_params;
  Perfc perfc;
  std::unique_ptr<TraceRing> trace;
  std::recursive_mutex mu;
  LockProfile lockprof;  // xenlockprof analog for `mu`
  // API callers blocked on `mu`.  The dispatcher hands the lock off while it
  // is behind schedule; otherwise a host too slow for the timer periods
  // (sanitizer builds, oversubscribed CPUs) would starve every API call.
  std::atomic<int> api_waiters_{0};
  int lock_depth_ = 0;  // recursion depth of `mu` (only touched with `mu` held)
  // RAII for C ABI entries: profiles the outermost acquisition.
  struct ApiLock {
    Engine* e;
    uint64_t t_acq = 0;
    bool outer = false;
    explicit ApiLock(Engine* x) : e(x) {
      if (e->mu.try_lock()) {
        take(false, 0);
        return;
      }
      const uint64_t t0 = LockProfile::clock_ns();
      e->api_waiters_.fetch_add(1, std::memory_order_relaxed);
      e->mu.lock();
      e->api_waiters_.fetch_sub(1, std::memory_order_relaxed);
      take(true, LockProfile::clock_ns() - t0);
    }
    void take(bool blocked, uint64_t wait_ns) {
      outer = e->lock_depth_++ == 0;
      if (outer) {
        e->lockprof.acquired(blocked, wait_ns);
        t_acq = LockProfile::clock_ns();
      }
    }
    ~ApiLock() {
      if (outer) e->lockprof.released(LockProfile::clock_ns() - t_acq);
      e->lock_depth_--;
      e->mu.unlock();
    }
    ApiLock(const ApiLock&) = delete;
    ApiLock& operator=(const ApiLock&) = delete;
  };

  std::vector<std::unique_ptr<Partition>> parts;
  std::vector<std::unique_ptr<Slot>> slots;
  std::vector<std::unique_ptr<Tenant>> tenants;
  std::vector<std::unique_ptr<Pool>> pools;

  gpbs_counter_ops_t counter_ops{};
  gpbs_actuator_ops_t actuator_ops{};
  bool dirty_actuation = false;
  // Per-GPU backend multiplexer (gpbs_backend_mux_add): one engine spanning
  // several GPUs drives one actuator + counter backend per GPU.  Backend i
  // serves partitions [lo, hi).
  struct MuxEntry {
    int lo, hi;
    gpbs_actuator_ops_t act;
    gpbs_counter_ops_t ctr;
  };
  std::vector<MuxEntry> mux;

  // --- time & timers (X:xen/common/timer.c analog) ---
  int64_t now() const;
  int timer_init(std::function<void(int64_t)> fn);
  void timer_set(int id, int64_t when);
  void timer_stop(int id);
  void timer_kill(int id);
  bool timer_armed(int id) const;
  int64_t next_deadline() const;
  void run_due(int64_t now);  // process timers and softirqs
  void raise_softirq(int part);
  void process_softirqs();
  void flush_actuation();

  // --- lifecycle ---
  int partition_add(int gpu, int xcd, int ctx = 0);
  int pool_create(const std::string& name, const std::string& sched);
  int pool_destroy(int pool);
  int pool_assign(int pool, int part);
  int pool_unassign(int pool, int part);
  int tenant_create(const std::string& name, int pool, int nslots, int weight, int cap);
  int tenant_destroy(int t);
  int tenant_move(int t, int pool);
  int tenant_set_nslots(int t, int n);

  // --- generic vcpu ops (schedule.c) ---
  bool runnable(const Slot& v) const;
  void runstate_change(Slot& v, Runstate rs, int64_t now);
  void vcpu_wake(Slot& v);
  void vcpu_sleep_nosync(Slot& v);
  void vcpu_block(Slot& v);
  void vcpu_unblock(Slot& v);
  void vcpu_pause(Slot& v);
  void vcpu_unpause(Slot& v);
  void vcpu_migrate(Slot& v);
  void schedule(int part);
  void context_saved(Slot& prev);
  void pmu_refresh(Slot& v);

  Scheduler* sched_of_part(int part);
  Scheduler* sched_of_tenant(int t);
  Tenant* tenant(int id) { return (id >= 0 && id < (int)tenants.size()) ? tenants[id].get() : nullptr; }
  Slot* slot(int id) { return (id >= 0 && id < (int)slots.size()) ? slots[id].get() : nullptr; }
  Pool* pool(int id) { return (id >= 0 && id < (int)pools.size()) ? pools[id].get() : nullptr; }
  Slot& curr_of(int part) { return *slots[parts[part]->curr]; }

  // --- observability ---
  void printk(const std::string& s);
  std::string dmesg(bool clear);
  std::string debug_keys(const std::string& keys);
  std::string dump_runq();      // 'r'
  std::string dump_domains();   // 'q'
  std::string dump_customized();// 'z' (P5)
  std::string check_invariants();
  void emit(uint32_t ev, uint32_t cpu, uint32_t a0 = 0, uint32_t a1 = 0, uint32_t a2 = 0, uint32_t a3 = 0) {
    trace->emit(now(), ev, cpu, a0, a1, a2, a3);
  }

  // --- fault injection (S13; GPBS_FAULT="kind=ppm[:param],...") ---
  // Each kind fires with probability ppm / 1e6 at its injection point, from a
  // seeded xorshift stream (reproducible runs): counter_drop (slot counters
  // not refreshed: stale vPMU), counter_reset (slot counters zeroed: a PMU
  // reset, exercises the Q5 skip), heartbeat_drop (tenant heartbeats lost),
  // actuate_delay (a flush of partition switches held back to the next
  // batch), timer_jitter (a due timer fires `param` us late).
  // rank_hang (the gang epoch thread of this rank stalls `param` ms before
  // its collective: exercises the other ranks' gang deadline) and torn_page
  // (a control-page publish pauses `param` us half-written: exercises the
  // tenants' seqlock retry) fire at injection points outside the engine,
  // through gpbs_fault_fire.
  enum FaultKind {
    F_COUNTER_DROP = 0, F_COUNTER_RESET, F_HEARTBEAT_DROP, F_ACTUATE_DELAY, F_TIMER_JITTER, F_RANK_HANG, F_TORN_PAGE,
    F_NKIND
  };
  uint32_t fault_ppm[F_NKIND] = {};
  int64_t fault_param[F_NKIND] = {};
  uint64_t fault_hits[F_NKIND] = {};
  uint64_t fault_rng = 0x9E3779B97F4A7C15ull;
  bool fault(int k) {
    if (!fault_ppm[k]) return false;
    fault_rng ^= fault_rng << 13;
    fault_rng ^= fault_rng >> 7;
    fault_rng ^= fault_rng << 17;
    if (fault_rng % 1000000u >= fault_ppm[k]) return false;
    fault_hits[k]++;
    perfc.incr(PC_fault_injected);
    return true;
  }
  int fault_parse(const char* spec);

  // --- dispatcher thread (real clock) ---
  int start();
  int stop();
  void kick();
  void heartbeat_check(int64_t now);
  int watchdog(int tenant, uint32_t id, uint32_t timeout_ms);
  void watchdog_fire(int tenant, int id);
  void watchdog_kill(Tenant& t);
  void classify_tick(int64_t now);
  void place_tenant_class(Tenant& t, Pool& pl, int layout);
  void budget_layout(Pool& pl, int64_t now, bool force);
  void place_budget(Tenant& t, Pool& pl, uint32_t ctx_mask, int stagger, uint32_t xcd_mask = 0);
  void place_parts(Tenant& t, Pool& pl, const Mask& m);
  void set_affinity(Slot& v, const Mask& m, int home = -1);
  void place_class(Slot& v, const Mask& m, int home);
  void send_home(Slot& v);

  int64_t sim_now = 0;

 private:
  struct TimerEnt {
    std::function<void(int64_t)> fn;
    uint64_t gen = 0;
    int64_t when = 0;
    bool armed = false;
    bool alive = false;
  };
  struct HeapEnt {
    int64_t when;
    uint64_t seq;
    int id;
    uint64_t gen;
    bool jittered = false;
    bool operator>(const HeapEnt& o) const { return when != o.when ? when > o.when : seq > o.seq; }
  };
  std::vector<TimerEnt> timers_;
  std::vector<int> free_timers_;
  std::priority_queue<HeapEnt, std::vector<HeapEnt>, std::greater<HeapEnt>> heap_;
  uint64_t seq_ = 0;
  bool in_softirq_ = false;
  std::string console_;
  std::thread thread_;
  std::condition_variable_any cv_;
  bool running_ = false;
  std::atomic<bool> kicked_{false};  // read lock-free by the final-approach spin
  int hb_timer_ = -1;
  int class_timer_ = -1;
  void loop();
};

}  // namespace gpbs
