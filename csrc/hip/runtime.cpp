// GPU runtime of gpbs on one MI355X (one process per GPU):
//
//  * GpuCtx     partition table (pinned, fine-grained host memory that tenant
//               kernels poll with system-scope loads; optional device copy
//               refreshed by k_partition_switch), per-(tenant,XCD) counter
//               blocks in HBM, a high-priority scheduler stream, and the
//               engine hooks: the actuator (context switch -> owner table) and
//               the counter backend (device counter_reduce + adapt kernels).
//  * Runner     a native tenant worker thread: it keeps up to `depth` units of
//               its workload in flight on its own HIP stream, launching only
//               while its tenant owns an XCD, relaunching revoked units, and
//               tells the engine when it has work (slot wake) and when it
//               drains (slot block).  This is the in-process tenant shim; the
//               cross-process one is pbs_amd/runtime/tenant.py over ctl pages.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <x86intrin.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../include/gpbs/gpbs.h"
#include "common.hpp"
#include "hwc_attr.h"

using namespace gpbs_hip;

extern "C" {
int gpbs_adapt_update(gpbs_adapt_state_t*, const gpbs_adapt_params_t*, uint64_t, uint64_t, uint64_t, uint64_t);
int gpbs_hip_gemm_units(int, int);
int gpbs_hwc_sample(uint64_t* out, int nxcd);
int gpbs_hwc_sample_se(uint64_t* se_out, uint64_t* x_out);
int gpbs_hwc_slot_per_se(int k);
int gpbs_hwc_active(void);
int gpbs_hip_gemm_bf16(const void*, const void*, void*, int, int, int, void*, const void*, unsigned, unsigned, void*,
                       void*, int, hipStream_t);
int gpbs_hip_stream_copy(const void*, void*, unsigned long long, unsigned, void*, const void*, unsigned, unsigned,
                         void*, void*, int, hipStream_t);
int gpbs_hip_reduce_bf16(const void*, const void*, void*, unsigned long long, unsigned, void*, const void*, unsigned,
                         unsigned, void*, void*, int, hipStream_t);
int gpbs_hip_gemv_bf16(const void*, const void*, void*, int, int, void*, const void*, unsigned, unsigned, void*, void*,
                       int, hipStream_t);
int gpbs_hip_partition_switch(void*, unsigned, const unsigned*, hipStream_t);
int gpbs_hip_counter_reduce(void*, void*, const int*, int, void*, hipStream_t);
int gpbs_hip_adapt(void*, const void*, const void*, const void*, int, const gpbs_adapt_params_t*, int*, hipStream_t);
int gpbs_hip_switch_probe(const void*, int, unsigned*, int, unsigned, unsigned long long, hipStream_t);
int gpbs_hip_hwc_attribute(const void*, void*, void*, void*, hipStream_t);
int gpbs_hip_hwc_attribute2(const void*, void*, void*, void*, hipStream_t, int);
int gpbs_hip_allreduce(const void*, unsigned, unsigned long long, unsigned, void*, const void*, unsigned, unsigned,
                       void*, void*, int, unsigned long long, unsigned long long, hipStream_t);
int gpbs_hip_gang_desc_size(void);
int gpbs_hip_gang_exchange(const void*, unsigned, const void*, void*, void*, unsigned long long, hipStream_t);
int gpbs_hip_coll_desc_size(void);
}

namespace {

// roctx ranges/marks: scheduler decisions next to tenant kernels
// on a rocprofv3 --marker-trace timeline.  Ranges (metric tick, counter
// sample, table publish) are always emitted -- a no-op call without a tool;
// per-switch marks format a string, so they need GPBS_ROCTX=1.
bool roctx_switch_marks() {
  static const bool on = [] {
    const char* v = std::getenv("GPBS_ROCTX");
    return v && std::atoi(v) > 0;
  }();
  return on;
}

struct RoctxRange {
  explicit RoctxRange(const char* m) { roctxRangePushA(m); }
  ~RoctxRange() { roctxRangePop(); }
};

int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// ---- table mode 2: the partition table in VRAM, written by the host ----
// A fine-grained VRAM allocation from the GPU agent's memory pool, made
// accessible to the CPU agent (hsa_amd_agents_allow_access): the host stores
// the owner words and then the epoch straight through the large-BAR mapping
// (write-combined, so each group is fenced), and tenant kernels poll it with
// agent-scope loads.  No kernel and no queue sits between a decision and the
// workgroups: measured on MI355X, host store -> device sees -> host sees the
// device's ack in 2.3 us (scripts/bar_probe.hip), where the k_partition_switch
// path needs a dispatch that waits for a free wave slot behind the tenants'
// persistent grids (37 us mean, 233 us max under the flagship co-run,
// profiles/rocprof_flagship_r2s5_summary.txt).
struct BarFind {
  uint32_t bdf = 0;
  hsa_agent_t gpu{}, cpu{};
  hsa_amd_memory_pool_t pool{};
  bool gpu_ok = false, cpu_ok = false, pool_ok = false;
};

hsa_status_t bar_pool_cb(hsa_amd_memory_pool_t p, void* ud) {
  auto* F = (BarFind*)ud;
  hsa_amd_segment_t seg;
  uint32_t fl = 0;
  if (hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
  if ((fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !F->pool_ok) {
    F->pool = p;
    F->pool_ok = true;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t bar_agent_cb(hsa_agent_t a, void* ud) {
  auto* F = (BarFind*)ud;
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !F->cpu_ok) {
    F->cpu = a;
    F->cpu_ok = true;
  } else if (t == HSA_DEVICE_TYPE_GPU && !F->gpu_ok) {
    uint32_t bdf = 0;
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
    if ((bdf & ~7u) == F->bdf) {  // this process's GPU (bus, device; any function)
      F->gpu = a;
      F->gpu_ok = true;
      hsa_amd_agent_iterate_memory_pools(a, bar_pool_cb, F);
    }
  }
  return HSA_STATUS_SUCCESS;
}

// Any size (the counter block too); zeroed through the mapping.
void* finegrained_alloc(int device, size_t bytes) {
  int bus = 0, dev = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess)
    return nullptr;
  BarFind F;
  F.bdf = ((uint32_t)bus << 8) | ((uint32_t)dev << 3);
  hsa_iterate_agents(bar_agent_cb, &F);
  if (!F.gpu_ok || !F.cpu_ok || !F.pool_ok) return nullptr;
  void* p = nullptr;
  bytes = (bytes + 4095) & ~(size_t)4095;
  if (hsa_amd_memory_pool_allocate(F.pool, bytes, 0, &p) != HSA_STATUS_SUCCESS) return nullptr;
  hsa_agent_t both[2] = {F.gpu, F.cpu};
  if (hsa_amd_agents_allow_access(2, both, nullptr, p) != HSA_STATUS_SUCCESS) {
    hsa_amd_memory_pool_free(p);
    return nullptr;
  }
  volatile uint64_t* w = (volatile uint64_t*)p;
  for (size_t i = 0; i < bytes / 8; ++i) w[i] = 0;
  _mm_sfence();
  return p;
}

// Host read of counter rows that the GPU keeps in fine-grained VRAM (round
// 6): SSE4.1 streaming loads pull a whole 64-byte line
// per PCIe read from the uncached BAR mapping, so the sampler's per-tick read
// of the active tenants' rows (~2 KiB) costs tens of us of one host thread
// and no GPU queue work -- no copyBuffer blit kernel on the tenants' CUs.
__attribute__((target("sse4.1"))) void bar_read(const void* src, void* dst, size_t bytes) {
  const __m128i* s = (const __m128i*)src;
  __m128i* d = (__m128i*)dst;
  for (size_t i = 0; i < bytes / 16; ++i) _mm_storeu_si128(d + i, _mm_stream_load_si128(const_cast<__m128i*>(s + i)));
  _mm_mfence();
}

// Host write into fine-grained VRAM through the BAR: non-temporal 16-byte
// stores out of the write-combining buffers, fenced before the launch that
// reads them.
__attribute__((target("sse4.1"))) void bar_store(void* dst, const void* src, size_t bytes) {
  __m128i* d = (__m128i*)dst;
  const __m128i* s = (const __m128i*)src;
  for (size_t i = 0; i < (bytes + 15) / 16; ++i) _mm_stream_si128(d + i, _mm_loadu_si128(s + i));
  _mm_sfence();
}

PartTable* bar_alloc(int device) {
  int bus = 0, dev = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess)
    return nullptr;
  BarFind F;
  F.bdf = ((uint32_t)bus << 8) | ((uint32_t)dev << 3);
  hsa_iterate_agents(bar_agent_cb, &F);
  if (!F.gpu_ok || !F.cpu_ok || !F.pool_ok) return nullptr;
  void* p = nullptr;
  if (hsa_amd_memory_pool_allocate(F.pool, 4096, 0, &p) != HSA_STATUS_SUCCESS) return nullptr;
  hsa_agent_t both[2] = {F.gpu, F.cpu};
  if (hsa_amd_agents_allow_access(2, both, nullptr, p) != HSA_STATUS_SUCCESS) {
    hsa_amd_memory_pool_free(p);
    return nullptr;
  }
  // Pool memory is not zeroed: clear the whole 4 KiB (a stale hold word
  // would stall every GATE_HOLD grab until the first latency unit completes)
  volatile u32* w = (volatile u32*)p;
  for (int i = 0; i < 1024; ++i) w[i] = 0;
  _mm_sfence();
  return (PartTable*)p;
}

// Owner words first, then the epoch, each group fenced out of the CPU's
// write-combining buffers (a kernel that sees the new epoch sees the owners).
void bar_write(PartTable* b, const u32* owners, u32 epoch);

// Whole-table resync from the host table (entering BAR mode): flags and the
// hold word too, not only the owners.
void bar_sync(PartTable* b, const PartTable* h) {
  *(volatile u32*)&b->flags = __atomic_load_n(&h->flags, __ATOMIC_ACQUIRE);
  *(volatile u32*)&b->hold = __atomic_load_n(&h->hold, __ATOMIC_ACQUIRE);
  bar_write(b, h->owner, __atomic_load_n(&h->epoch, __ATOMIC_ACQUIRE));
}

void bar_write(PartTable* b, const u32* owners, u32 epoch) {
  volatile u32* o = (volatile u32*)b->owner;
  for (int x = 0; x < kXcds * kCtx; ++x) o[x] = owners[x];
  _mm_sfence();
  *(volatile u32*)&b->epoch = epoch;
  _mm_sfence();
}

struct GpuCtx;
void set_hold(GpuCtx* c, u32 v);

struct GpuCtx {
  int device = 0;
  int part_base = 0;  // engine partition id of XCD 0
  int table_mode = 0; // 0: pinned host table, 1: device table + partition_switch kernel,
                      // 2: device table the host writes directly (BAR; no kernel, no queue)
  int spatial = 0;    // 1: the two partitions of an XCD are CU halves (GATE_SPATIAL)
  PartTable* h_table = nullptr;  // pinned host (device-visible)
  PartTable* d_table = nullptr;  // device copy (table_mode 1)
  PartTable* b_table = nullptr;  // host-writable VRAM table (table_mode 2), allocated on first use
  u64* d_cnt = nullptr;          // [kMaxTenants][kXcds][kNumPmc]
  bool cnt_bar = false;          // d_cnt lives in host-readable fine-grained VRAM (bar_read, no copy kernel)
  std::atomic<int> cnt_rows{1};  // rows [0, cnt_rows) can be non-zero: the largest runner tenant id + 1
  u64* d_prev = nullptr;
  u64* h_out = nullptr;          // pinned mapped: deltas [kMaxTenants][4]
  int* h_ids = nullptr;          // pinned mapped
  gpbs_adapt_state_t* h_states = nullptr;
  u64* h_spin = nullptr;         // [2][kMaxTenants]
  int* h_dirs = nullptr;
  u64* h_adelta = nullptr;        // adapt inputs (separate from the async reduce buffers)
  hipStream_t sched_stream = nullptr;
  gpbs_engine_t* engine = nullptr;
  int nctx = 1;                  // issue contexts per XCD in use (1..kCtx)
  int waveprio = 0;              // latency-class runners raise their wave priority
  // Latency lane: ungated latency-class runners (priority > 0) launch on a
  // stream CU-masked to this class half (0: SEs {0,1}, 1: SEs {2,3}; -1:
  // unmasked).  The memory half hosts small-footprint stream / reduce
  // workgroups a GEMV can co-reside with; on the compute half its
  // workgroups queue behind persistent GEMM workgroups holding the CUs' LDS
  // until a whole GEMM unit ends.
  int lat_half = -1;
  int hold_enable = 0;           // latency requests hold the memory-class tenants (GATE_HOLD)
  // Latency-request hold: count of latency units in flight and the hold
  // word derived from it, changed together under hold_mu.  hold_gen changes
  // whenever the hold is switched off (holds reset): a runner releases only
  // the raises it made in the current generation.
  std::mutex hold_mu;
  int holds = 0;
  uint64_t hold_gen = 0;
  std::atomic<uint64_t> hold_raises{0};
  // per-tenant contention class cache (-1 unknown), refreshed under the
  // engine lock by the metric tick and table publishes: launch() reads it
  // without taking the engine lock
  std::atomic<int> cls_cache[kMaxTenants];
  u32 pending[kXcds * kCtx];
  u32 epoch = 0;
  // async counter reduce (one metric period of lag, never blocks the engine)
  bool red_pending = false;
  int red_n = 0;
  int red_buf = 0;
  int* h_ids2 = nullptr;
  u64* h_out2 = nullptr;
  hipEvent_t red_ev = nullptr;
  // Live hardware counters (csrc/hip/hwc.cpp), attributed by OWNERSHIP (the
  // per-vCPU PMU save/restore of X:xen/arch/x86/pmustate.c:87-135 done in
  // space): a sampler thread snapshots, at one instant every period, the
  // cumulative per-(XCD, SE) and per-XCD hardware counters together with
  // the cumulative ns every tenant has owned every partition; the metric tick
  // (engine lock held) only does arithmetic on the newest snapshot pair.  A
  // synchronous device-counting sample costs ~0.2 ms, so it never runs under
  // the engine lock.  The modeled per-tile block is snapshotted alongside as
  // a cross-check (attribution error vs model), never as an input.
  int hwc = 0;
  int slot_se[kNumPmc] = {1, 1, 1, 0};  // slot k resolved per shader engine
  u64* h_blk = nullptr;                 // pinned landing buffer of d_cnt copies
  std::vector<u64> snap_blk, blk_prev;  // newest published / last consumed model block
  std::vector<u64> red_prev;            // modeled-counter mode: the block the last metric tick read
  std::vector<u64> snap_se;             // [kXcds * kCtx(=SEs) * kNumPmc]
  std::vector<u64> snap_x;              // [kXcds * kNumPmc]
  std::vector<int64_t> snap_own;        // [kMaxTenants * kXcds * kCtx]
  uint64_t snap_seq = 0, used_seq = 0;
  bool hw_primed = false;
  // Attribution of a snapshot (csrc/hip/hwc_attr.h): on the host by default
  // (round 6: hwc_attr_host, a few us of the metric tick, and no kernel that
  // waits for a wave slot behind the tenants' persistent grids -- 40-60 us
  // mean, 200-440 us max per k_hwc_attribute on a full GPU,
  // profiles/r6/s13_*); param device_attr 1: k_hwc_attribute on the
  // scheduler stream, launched by one metric tick and harvested by the next.
  int dev_attr = 0;
  HwcAttrPrev hst;                  // host path state
  HwcAttrIn* h_ain = nullptr;       // pinned: the snapshot the metric tick fills
  HwcAttrIn* d_ain = nullptr;       // device staging copy the kernel reads
  HwcAttrIn* f_ain = nullptr;       // fine-grained VRAM copy the host writes through the BAR (no blit)
  HwcAttrOut* h_aout = nullptr;     // pinned mapped, written by the kernel
  HwcAttrPrev* d_ast = nullptr;     // device-resident previous snapshot
  hipEvent_t attr_ev = nullptr;
  bool attr_pending = false;
  uint64_t attr_launches = 0, attr_busy_skips = 0, attr_host = 0;
  // in-run cost of k_hwc_attribute, from its own 100 MHz entry / exit stamps,
  // and launch -> harvest latency (the metric period it lags by)
  uint64_t attr_harvested = 0, attr_ticks_sum = 0, attr_ticks_max = 0;
  int64_t attr_launch_ns = 0, attr_lag_sum_ns = 0;
  hipEvent_t blk_ev = nullptr;
  hipStream_t hwc_stream = nullptr;
  std::thread hwc_th;
  std::atomic<bool> hwc_stop{false};
  std::mutex snap_mu;
  int hwc_period_us = 1000;
  // Adaptive sampling: every device-counting sample perturbs the tenants
  // (measured on MI355X: two GEMM tenants 1.09 solo-equivalents sampled every
  // 1 ms, 1.23 every 4 ms, 1.23 every 10 ms; none 1.25-1.27 without a
  // sampler, profiles/corun_r2/hwc_period.md).  While the partition table is
  // changing (time-sharing, re-placement) the sampler runs every
  // hwc_period_us, so exclusive-ownership windows stay short; once no owner
  // has changed for 20 ms it backs off to hwc_slow_us.
  // Round 3: with the lean counter set a 1 ms sample costs a GEMM ~0.75 %
  // (scripts/hwc_cost.py), so the sampler keeps the reference's 1 ms period
  // (CSCHED_METRIC_TICK_PERIOD, X:xen/common/sched_credit.c:55) and no longer
  // backs off; param slow_us 4000 restores the round-2 back-off.
  // Round 4: back off to 50 ms once no owner has changed for 20 ms (phase
  // triggers still open 1 ms bursts): config #5 1.2343 vs 1.2249 (the shim
  // tenants' layout is steady; profiles/r4/llm5_backoff_s22.txt), runner mixes
  // equal or +0.003 with a quarter of the samples on steady layouts
  // (sampler_backoff_s23.txt).  0: never back off.
  int hwc_slow_us = 50000;  // param slow_us
  // Duty-cycle cap: a sample stalls the command processor for its duration
  // (every counter record is a register read it performs), and what that
  // costs the tenants varies from box to box (145-190 us per lean sample on
  // one MI355X, ~500 us on another: scripts/hwc_cost.py).  The period
  // stretches so that sampling takes at most hwc_duty_pct % of the time
  // (EWMA of the sample duration); 0 disables the cap.
  // Measured on the 4-tenant mix: a 25 % duty (lean set, 1.15 ms) cost the
  // flagship 5 % of its aggregate, 5 % duty (4 ms) 0.5 %.
  int hwc_duty_pct = 1;  // param duty_pct (profiles/r3: 5 % costs 0.01 of 4mix aggregate, 2 % 0.004, 1 % none measurable)
  int hwc_burst_ms = 20;  // param burst_ms: 1 ms hardware sampling after a trigger
  // Sample budget (round 4): a token bucket over EVERY hardware sample,
  // bursts included -- the round-3 bursts re-armed back to back in
  // time-shared regions (every quantum is an owner change: 1539 samples per
  // 8mix run).  Tokens accrue so that samples take at most hwc_budget_pct %
  // of the time on average (EWMA sample time), up to hwc_bucket samples
  // banked; a burst tick without a token is skipped.  0: no budget.
  int hwc_budget_pct = 5;    // param budget_pct
  int hwc_bucket = 50;       // param bucket: a phase change's burst plus a flip back
  double hwc_tokens = 50;
  int64_t hwc_tok_ns = 0;
  uint64_t hwc_denied = 0;   // burst ticks skipped for lack of a token
  // Switch-aligned sampling (round 5; the per-vCPU PMU save at every context
  // switch, X:xen/arch/x86/domain.c:1600,1619 -> perfctr.c:1547-1572): every
  // table publish that changes an owner records, per partition, when it
  // changed and the quantum the new owner was given, and wakes the sampler.
  // The sampler takes a hardware sample one drain guard after the switch --
  // the revoked workgroups have left the partition, the new owner's tenure
  // starts -- so sample intervals coincide with tenures and a time-shared
  // tenant's window is clean (csrc/hip/hwc_attr.h, `drained`).  Which switches
  // get a sample, under the token budget:
  //   * one that ends a tenure whose start was sampled (closes a window);
  //   * one that starts a tenure of at least hwc_long_us (opens a window:
  //     memory-class quanta, 11 ms in the MI355X profile);
  //   * a short tenure (compute quanta, 1 ms) opens a window -- a sample pair,
  //     the second one ahead of the quantum's end -- about once per
  //     hwc_pair_gap_us (jittered, so co-sharers rotating in lockstep all get
  //     measured) when the bucket holds the pair plus a reserve.
  int hwc_align = 1;          // switch-aligned samples on
  int hwc_guard_us = 150;     // publish -> sample: a revoked GEMM tile / stream chunk drains in ~50-150 us
  int hwc_long_us = 3000;     // tenures at least this long open a window at every switch
  int hwc_pair_gap_us = 20000;  // short tenures: about one measured pair per this long
  int64_t part_chg_ns[kXcds * kCtx] = {};  // publish time of each partition's last owner change (mu)
  u32 q_pending[kXcds * kCtx] = {};        // quantum (us) of the owner each pending entry names (mu)
  u32 part_q_us[kXcds * kCtx] = {};        // ... as published (mu)
  u32 sw_changed = 0;                      // partitions changed since the sampler consumed them (mu)
  // the last tenant (not kNoOwner) each partition was handed to (mu): a
  // partition that goes idle and comes back to the same tenant (a torch
  // tenant blocking between its 6 ms decode slices) did not change owner for
  // the sampler -- nothing runs while it is idle
  u32 last_real[kXcds * kCtx];
  int64_t sw_first_p[kXcds * kCtx] = {};   // per pending partition: its first change since (mu)
  int64_t sw_last_ns = 0;                  // latest publish that changed an owner (mu)
  std::vector<int64_t> snap_chg;           // part_chg_ns at the newest snapshot (snap_mu)
  int64_t snap_t = 0;                      // its sample time (snap_mu)
  std::vector<int64_t> used_chg;           // ... of the last consumed snapshot (snap_mu)
  int64_t used_t = 0;
  std::vector<int64_t> own_prev;           // owned ns at the last consumed snapshot (host copy, snap_mu)
  uint64_t align_samples = 0, align_close = 0, align_long = 0, align_short = 0, align_denied = 0;
  int64_t ts_gap_sum = 0;                  // sample-to-sample gaps over intervals with a switch (time-shared)
  uint64_t ts_gaps = 0;
  // Model fallback (default on): a tenant that ran substantially in an
  // interval without a clean window, and whose last clean window is older
  // than hwc_stale_us (250 ms), reports the interval's MODELED deltas scaled per
  // counter by its hardware/model ratio from its own clean windows (EWMA);
  // uncalibrated, the period reports nothing.  Otherwise such a period is
  // skipped (the PBS idle-sample rule), and a sliver -- a tenant that held
  // its partitions for less than (100 - clean_pct) % of the interval, the
  // edge of a neighbouring tenure -- never counts.
  int model_fallback = 1;
  int hwc_stale_us = 250000;
  // 1 ms metric cadence (round 6; param cadence, default
  // on): every metric tick a calibrated tenant reports its MODELED deltas of
  // that tick scaled per counter by its hardware/model ratio, and each clean
  // hardware window re-anchors the ratio instead of reporting (it already
  // did, tick by tick); a tenant not calibrated yet reports its clean
  // windows as before.  The reference reads its PMU every 1 ms
  // (X:xen/common/sched_credit.c:55,450-465).
  int model_cadence = 1;
  std::vector<u64> cad_prev;                   // the block at the previous tick (snap_mu)
  bool cad_primed = false;
  uint64_t t_model[kMaxTenants] = {};          // metric periods delivered from the calibrated model
  uint64_t t_moved[kMaxTenants] = {};          // ticks its modeled counters moved (calibrated or not)
  uint64_t cad_calls = 0;                      // cadence ticks
  int64_t cad_dbg[512][3] = {};                // debug ring: tick time, tenant 1 / 2 instruction sums
  uint64_t t_delivered[kMaxTenants] = {};      // metric periods with any delivery (clean, fallback, model)
  int64_t t_first_ns[kMaxTenants] = {}, t_last_ns[kMaxTenants] = {};  // first / last delivery (period stats)
  double mod_cur[kMaxTenants][kNumPmc] = {};       // modeled deltas of the newest consumed snapshot
  double mod_inflight[kMaxTenants][kNumPmc] = {};  // ... of the snapshot whose attribution is in flight
  double pres_cur[kMaxTenants] = {};               // largest owned share of a partition over the interval
  double pres_inflight[kMaxTenants] = {};
  int64_t t_inflight = 0;                          // sample time of the in-flight attribution
  double cal[kMaxTenants][kNumPmc] = {};           // hardware / model per counter (0: not calibrated)
  int64_t last_clean_ns[kMaxTenants] = {};
  // Measurement tenures: a tenant that ran without a clean window for
  // hwc_measure_ms asks the engine (gpbs_tenant_measure) for one tenure of
  // long_us + the drain guard + two sample times on some partition -- the
  // switch-aligned long window then covers it.  Tenants on 1 ms quanta
  // (compute-bound, at min_us) otherwise get clean windows only from the
  // budgeted short pairs, which the host table's 550 us guard mostly leaves
  // as slivers (s10 8mix: GEMM tenants clean in 0.16-0.39 of their periods).
  int hwc_measure_ms = 40;
  int64_t last_ran_ns[kMaxTenants] = {};   // last interval the tenant ran in (snap_mu)
  int64_t measure_req_ns[kMaxTenants] = {};
  uint64_t measure_reqs = 0;
  uint64_t fallback_periods = 0, clean_periods = 0, skipped_periods = 0, sliver_periods = 0;
  uint64_t t_clean[kMaxTenants] = {}, t_fallback[kMaxTenants] = {}, t_skipped[kMaxTenants] = {},
           t_sliver[kMaxTenants] = {};
  int hwc_watch = 1;      // param watch: read the modeled block every tick (the burst trigger)
  int64_t hwc_next_period_ns = 1000000;
  std::atomic<uint64_t> hwc_triggers{0};
  uint64_t hwc_burst_samples = 0;
  double hwc_dt_ewma = 0;
  int64_t hwc_period_sum_ns = 0;
  std::atomic<uint64_t> hwc_slow_samples{0};
  int64_t hwc_ns = 0, hwc_ns_max = 0;
  uint64_t hwc_samples = 0;
  double hw_sum[kNumPmc] = {}, model_sum[kNumPmc] = {};  // attributed vs modeled totals
  double unatt[kNumPmc] = {};                             // hardware counts no owner explains
  double metric_sum[kNumPmc] = {};                        // counts delivered to the PBS metric (clean windows)
  // exclusive-ownership window: min % of an interval one owner must hold (0:
  // pro rata).  80: a switch-aligned 1 ms compute tenure keeps ~85 % of its
  // interval (the next tenure's first drain guard closes it).
  int clean_pct = 80;
  double att_total[kMaxTenants][kNumPmc] = {};            // per-tenant attributed hardware totals
  double met_total[kMaxTenants][kNumPmc] = {};            // per-tenant totals that reached the PBS metric
  double mod_total[kMaxTenants][kNumPmc] = {};            // per-tenant modeled totals (cross-check)
  u64 last_delta[kMaxTenants][kNumPmc];
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<uint64_t> switches{0}, flushes{0}, metric_calls{0};
  int64_t metric_ns = 0;
  // ownership accounting: cumulative ns each tenant held each partition
  // (xcd * kCtx + ctx), and the base the ownership() query subtracts
  int64_t own_ns[kMaxTenants][kXcds * kCtx];
  int64_t own_base[kMaxTenants][kXcds * kCtx];
  int64_t last_pub_ns = 0;
  std::atomic<int64_t> revoke_ns[kMaxTenants] = {};  // last publish that took a partition from the tenant
  std::atomic<int64_t> grant_ns[kMaxTenants] = {};   // last publish that gave the tenant a partition
  // Per-tenant switch cost (round 6; the runners measure it, the sampler
  // thread hands it to the engine as the tenant's quantum floor basis):
  // EWMA (1/8) of the revocation drain -- publish that took a partition ->
  // the interrupted unit's grid has left (co-sharers of a region share one
  // queue, so the next owner's grid starts only then) -- and of the re-entry
  // ramp -- publish that gave a partition back -> the tenant's next launch.
  std::atomic<int64_t> swc_drain_ns[kMaxTenants] = {}, swc_ramp_ns[kMaxTenants] = {};
  std::atomic<uint64_t> swc_drain_n[kMaxTenants] = {}, swc_ramp_n[kMaxTenants] = {};
  int64_t swc_pushed_ns[kMaxTenants] = {};  // sampler thread: the cost last given to the engine
  hipEvent_t adapt_ev = nullptr;  // device adapt: bounded poll, never a blocking sync
  bool adapt_pending = false;
  // Asynchronous device adapt (engine adapt_launch / adapt_harvest): pinned
  // buffer sets; a launch uses a free one, the next tick of the SAME pool
  // harvests it (matched by its tenant ids: pools sharing this context never
  // see each other's results).  A launch nobody harvested within kAbufOrphan
  // later launches (its engine stopped, or its pool went away) is freed once
  // its kernel is done.
  static constexpr int kAbuf = 6;
  static constexpr uint64_t kAbufOrphan = 8;
  struct AdaptBuf {
    gpbs_adapt_state_t* st = nullptr;  // in/out, pinned mapped
    u64* delta = nullptr;              // [kMaxTenants][4]
    u64* spin = nullptr;               // [2][kMaxTenants]
    int ids[kMaxTenants];
    int n = 0;
    int state = 0;  // 0 free, 1 pending, 2 pending + result discarded
    uint64_t gen = 0;  // async_launches at its launch
    hipEvent_t ev = nullptr;
  } abuf[kAbuf];
  uint64_t async_launches = 0, async_late = 0, async_busy = 0;
  uint64_t adapt_late = 0, adapt_calls = 0, adapt_busy = 0;
  int se_mode = 0;  // partitions are exclusive shader engines (GATE_SE)
  // Class-share mode (SE mode): when every tenant holding partitions is of
  // ONE contention class, runners launch ungated full-GPU grids (co-resident:
  // two GEMMs fill each other's MFMA stalls) except in periodic exclusive
  // probe windows that keep the per-tenant counters measurable (attribution
  // skips shared intervals).  Opt-in: it was written against a misaligned
  // split (0.73); with co-class tenants on aligned SE halves and the
  // adaptive sampler the split measured 1.253 vs 1.240 shared (none 1.252).
  int share_enable = 0;
  std::atomic<int> share{0};
  int64_t share_ns = 0, share_since = 0;  // cumulative shared time (sampler thread)
  uint64_t share_tick = 0;
  int probe_every = 40, probe_len = 4;  // params probe_every / probe_len (every 0: no probe windows)
  int64_t snap_share = 0, share_prev = 0, share_base = 0;
  int muxed = 0;    // ops installed through the engine's backend mux
};

// Cumulative ownership ns of every (tenant, partition) up to now, including
// the interval since the last table change.  Caller holds c->mu.
void own_snapshot_locked(const GpuCtx* c, int64_t* out) {
  const int64_t t = mono_ns();
  std::memcpy(out, c->own_ns, sizeof(c->own_ns));
  if (!c->last_pub_ns) return;
  for (int x = 0; x < kXcds * kCtx; ++x) {
    const u32 o = c->h_table->owner[x] & kOwnerMask;
    if (o < (u32)kMaxTenants) out[o * kXcds * kCtx + x] += t - c->last_pub_ns;
  }
}

// ---------------------------------------------------------------- engine hooks

void act_on_switch(void* user, int part, int, int next, int, int32_t quantum_us, int64_t) {
  GpuCtx* c = (GpuCtx*)user;
  const int i = part - c->part_base;
  if (i < 0 || i >= kXcds * c->nctx) return;
  const int x = i / c->nctx, ctx = i % c->nctx;
  {
    std::lock_guard<std::mutex> g(c->mu);
    c->pending[x * kCtx + ctx] = next >= 0 ? (u32)next : kNoOwner;
    c->q_pending[x * kCtx + ctx] = quantum_us > 0 ? (u32)quantum_us : 0u;
  }
  c->switches++;
  if (roctx_switch_marks()) {  // TRC_SCHED_SWITCH analog (X:xen/common/schedule.c:1138-1151)
    char m[64];
    std::snprintf(m, sizeof m, "gpbs:switch xcd%d.%d -> t%d", x, ctx, next);
    roctxMarkA(m);
  }
}

// Spatial mode: mark an XCD split when its two owners are of different
// contention classes (measured: CU-disjoint halves beat co-residence for
// compute + memory pairs; same-class pairs -- two GEMMs filling each other's
// kernel-boundary bubbles, two streams sharing HBM -- do better sharing the
// whole XCD, and a lone owner takes all of it: work conservation).
void mark_splits(GpuCtx* c) {
  for (int x = 0; x < kXcds; ++x) {
    u32& a = c->pending[x * kCtx];
    u32& b = c->pending[x * kCtx + 1];
    a &= kOwnerMask | (a == kNoOwner ? kSplitBit : 0u);
    b &= kOwnerMask | (b == kNoOwner ? kSplitBit : 0u);
    if (!c->spatial || c->nctx != 2 || a == kNoOwner || b == kNoOwner || a == b) continue;
    // No engine attached (manual tables): distinct owners are split.  The
    // class comes from the cache (c->mu is held: no engine lock from here,
    // the dispatcher takes them in the opposite order).
    const int ca = c->engine ? (a < (u32)kMaxTenants ? c->cls_cache[a].load(std::memory_order_relaxed) : -1) : 0;
    const int cb = c->engine ? (b < (u32)kMaxTenants ? c->cls_cache[b].load(std::memory_order_relaxed) : -1) : 1;
    if (ca >= 0 && cb >= 0 && ca != cb) {
      a |= kSplitBit;
      b |= kSplitBit;
    }
  }
}

// Publish the pending assignment.  Everything -- split marks, the change
// test, the host / BAR table stores and the k_partition_switch enqueue (from
// copies of pending and epoch) -- happens under c->mu, so two publishers (the
// dispatcher and an API caller) cannot interleave owner words in any table.
// publish_locked: caller holds c->mu; returns whether an owner changed.
bool publish_locked(GpuCtx* c) {
  mark_splits(c);
  bool changed = false;
  for (int x = 0; x < kXcds * kCtx; ++x)
    if (__atomic_load_n(&c->h_table->owner[x], __ATOMIC_RELAXED) != c->pending[x]) changed = true;
  if (!changed) return false;
  {
    const int64_t t = mono_ns();
    if (c->last_pub_ns)
      for (int x = 0; x < kXcds * kCtx; ++x) {
        const u32 o = c->h_table->owner[x] & kOwnerMask;
        if (o < (u32)kMaxTenants) c->own_ns[o][x] += t - c->last_pub_ns;
      }
    c->last_pub_ns = t;
    for (int x = 0; x < kXcds * kCtx; ++x) {
      const u32 o = c->h_table->owner[x] & kOwnerMask;
      if ((c->pending[x] & kOwnerMask) == o) continue;
      if (o < (u32)kMaxTenants) c->revoke_ns[o].store(t, std::memory_order_relaxed);
      const u32 nw = c->pending[x] & kOwnerMask;
      if (nw < (u32)kMaxTenants) c->grant_ns[nw].store(t, std::memory_order_relaxed);
      // switch-aligned sampling: when and to whom this partition changed --
      // an idle gap inside one tenant's tenure is no change (config #5: a
      // sample, 0.9 ms of command-processor stall with 12 hardware queues,
      // at every decode step ate the 5 % budget and ~3 % of both tenants)
      if (nw >= (u32)kMaxTenants || nw == c->last_real[x]) {
        if (nw < (u32)kMaxTenants) c->part_q_us[x] = c->q_pending[x];
        continue;
      }
      c->last_real[x] = nw;
      c->part_chg_ns[x] = t;
      c->part_q_us[x] = c->q_pending[x];
      if (!((c->sw_changed >> x) & 1u)) c->sw_first_p[x] = t;
      c->sw_changed |= 1u << x;
      c->sw_last_ns = t;
    }
    for (int x = 0; x < kXcds * kCtx; ++x) __atomic_store_n(&c->h_table->owner[x], c->pending[x], __ATOMIC_RELEASE);
    c->epoch++;
    __atomic_store_n(&c->h_table->epoch, c->epoch, __ATOMIC_RELEASE);
    if (c->table_mode == 2) bar_write(c->b_table, c->h_table->owner, c->epoch);
    if (c->table_mode == 1) {
      u32 own[kXcds * kCtx];
      std::memcpy(own, c->pending, sizeof(own));
      gpbs_hip_partition_switch(c->d_table, c->epoch, own, c->sched_stream);
    }
  }
  c->flushes++;
  return true;
}

void publish(GpuCtx* c) {
  RoctxRange rr("gpbs:publish");
  bool changed;
  {
    std::lock_guard<std::mutex> g(c->mu);
    changed = publish_locked(c);
  }
  if (changed) c->cv.notify_all();
}

// Refresh the class cache of every tenant (engine lock held by the caller).
void refresh_classes(GpuCtx* c) {
  if (!c->engine) return;
  for (int t = 0; t < kMaxTenants; ++t) c->cls_cache[t].store(gpbs_tenant_class(c->engine, t), std::memory_order_relaxed);
}

void act_on_flush(void* user, int64_t) {
  GpuCtx* c = (GpuCtx*)user;
  refresh_classes(c);
  publish(c);
}

// The hold word goes wherever the tenants read their table from: the pinned
// host table (always) and the BAR-written VRAM table whenever it exists (a
// later switch into BAR mode must not find a stale word).  Caller holds
// hold_mu (or has no concurrent hold users).
void set_hold(GpuCtx* c, u32 v) {
  __atomic_store_n(&c->h_table->hold, v, __ATOMIC_RELEASE);
  if (c->b_table) {
    *(volatile u32*)&c->b_table->hold = v;
    _mm_sfence();
  }
}

// A latency unit enters flight: count it; the first one raises the word.
// Returns the generation the raise belongs to.
uint64_t hold_acquire(GpuCtx* c) {
  std::lock_guard<std::mutex> g(c->hold_mu);
  if (c->holds++ == 0) {
    set_hold(c, 1);
    c->hold_raises.fetch_add(1, std::memory_order_relaxed);
  }
  return c->hold_gen;
}

// A latency unit left flight (completed, or its runner stopped): the last one
// clears the word.  Raises of an older generation (the hold was switched off
// and the count reset since) are ignored.
void hold_release(GpuCtx* c, uint64_t gen) {
  std::lock_guard<std::mutex> g(c->hold_mu);
  if (gen != c->hold_gen || c->holds <= 0) return;
  if (--c->holds == 0) set_hold(c, 0);
}

void act_on_park(void*, int, int, int) {}

// Counter backend, asynchronous: tick k harvests the reduce launched at tick
// k-1 (normally long finished) and launches the next one on the high-priority
// scheduler stream, so the engine lock is never held across a device sync.
// Every counted event is reported exactly once, one metric period late.
// Class-share decision (sampler thread, ~1 kHz): share while every distinct
// owner in the table is classified and of one class (>= 2 owners); every 40th
// decision opens a 4-decision exclusive probe window.
void share_update(GpuCtx* c) {
  int want = 0;
  if (c->share_enable && c->se_mode && c->engine) {
    int owners[kXcds * kCtx], n = 0;
    for (int x = 0; x < kXcds * kCtx; ++x) {
      const u32 o = __atomic_load_n(&c->h_table->owner[x], __ATOMIC_ACQUIRE) & kOwnerMask;
      if (o >= (u32)kMaxTenants) continue;
      bool seen = false;
      for (int k = 0; k < n && !seen; ++k) seen = owners[k] == (int)o;
      if (!seen) owners[n++] = (int)o;
    }
    if (n >= 2) {
      const int c0 = c->cls_cache[owners[0]].load(std::memory_order_relaxed);
      want = c0 >= 0;
      for (int k = 1; k < n && want; ++k) want = c->cls_cache[owners[k]].load(std::memory_order_relaxed) == c0;
    }
    if (want && c->probe_every > 0 && (c->share_tick++ % (uint64_t)c->probe_every) < (uint64_t)c->probe_len)
      want = 0;  // exclusive probe window
  }
  const int64_t t = mono_ns();
  const int was = c->share.load(std::memory_order_relaxed);
  if (was) c->share_ns += t - c->share_since;
  c->share_since = t;
  if (want != was) c->share.store(want, std::memory_order_release);
}

inline u64 dpos(u64 a, u64 b) { return a >= b ? a - b : 0; }  // Q5: a counter reset is no negative delta

// The drain guard in effect: hwc_guard_us covers a revoked tile / chunk
// (~50-150 us) once workgroups see the new owner word, which takes ~16 us on
// the device / BAR tables and ~340 us polling the pinned host table over
// PCIe (p50 for a 1024-workgroup grid, profiles/micro/microbench_r2.json).
int64_t guard_ns(const GpuCtx* c) {
  const int host = __atomic_load_n(&c->table_mode, __ATOMIC_ACQUIRE) == 0;
  return ((int64_t)c->hwc_guard_us + (host ? 400 : 0)) * 1000;
}

// The modeled counter block into `out` (kBlk u64): rows [0, cnt_rows) are
// read, the rest left as they were.  Fine-grained VRAM: CPU streaming loads
// through the BAR (no GPU queue work); device memory: a copy on hwc_stream.
bool read_block(GpuCtx* c, u64* out) {
  constexpr int kRow = kXcds * kNumPmc;
  if (c->cnt_bar) {
    const int rows = std::min(kMaxTenants, std::max(1, c->cnt_rows.load(std::memory_order_relaxed)));
    bar_read(c->d_cnt, out, sizeof(u64) * (size_t)rows * kRow);
    return true;
  }
  if (hipMemcpyAsync(c->h_blk, c->d_cnt, sizeof(u64) * kMaxTenants * kRow, hipMemcpyDeviceToHost, c->hwc_stream) !=
      hipSuccess)
    return false;
  hipEventRecord(c->blk_ev, c->hwc_stream);
  hipEventSynchronize(c->blk_ev);
  std::memcpy(out, c->h_blk, sizeof(u64) * kMaxTenants * kRow);
  return true;
}

// Sampler thread.  Every hwc_period_us (1 ms) it reads the modeled per-tile
// counter block (a 16 KiB device-to-host copy: no command-processor work) and
// watches each tenant's modeled miss rate; a HARDWARE sample -- which stalls
// the command processor for its duration and perturbs the tenants -- is taken
//   * one drain guard after a table publish that changed owners, when the
//     switch closes or opens a tenure window (switch-aligned, see GpuCtx);
//   * in a burst, every tick, for burst_ms after a tenant's modeled miss rate
//     moved by more than 3x (a phase change), so the classifier sees the
//     change at 1 ms resolution;
//   * otherwise when the duty-cycle cap allows (sample time <= hwc_duty_pct %
//     of the time), backing off to hwc_slow_us once no owner changed for
//     20 ms, which bounds what steady-state sampling costs.
// Every sample spends a token of the budget.  Classification and PBS
// decisions use the hardware counters; the modeled counters are the trigger
// and the calibrated fallback.
void hwc_loop(GpuCtx* c) {
  hipSetDevice(c->device);
  constexpr int kBlk = kMaxTenants * kXcds * kNumPmc;
  constexpr int kOwn = kMaxTenants * kXcds * kCtx;
  constexpr int P = kXcds * kCtx;
  std::vector<u64> blk(kBlk), se(kXcds * kCtx * kNumPmc), xs(kXcds * kNumPmc);
  std::vector<u64> watch_prev(kBlk, 0);
  std::vector<double> watch_rate(kMaxTenants, -1.0);
  std::vector<int64_t> own(kOwn), chg(P);
  roctxNameOsThread("gpbs-hwc-sampler");
  constexpr int64_t kSteadyNs = 20000000;  // slow_us back-off: no owner change for 20 ms
  uint64_t last_sw = c->flushes.load();
  int64_t last_change = mono_ns(), last_hw = 0, burst_until = mono_ns() + (int64_t)c->hwc_burst_ms * 1000000;
  int64_t next_tick = mono_ns(), seen_pub = 0, next_pair = 0;
  bool watch_primed = false, sw_since_hw = false, slow = false, burst = false;
  u32 open = 0;  // partitions whose current tenure began with a (switch-aligned) sample
  uint64_t rng = 0x2545F4914F6CDD1Dull;
  // one hardware sample plus the snapshot it belongs to; false if the read failed
  auto sample = [&](int64_t t0) -> bool {
    if (c->hwc_budget_pct > 0) c->hwc_tokens -= 1.0;
    RoctxRange rr("gpbs:hwc_sample");
    const int64_t s0 = mono_ns();
    const int rc = gpbs_hwc_sample_se(reinterpret_cast<uint64_t*>(se.data()), reinterpret_cast<uint64_t*>(xs.data()));
    {
      std::lock_guard<std::mutex> g(c->mu);
      own_snapshot_locked(c, own.data());
      chg.assign(c->part_chg_ns, c->part_chg_ns + P);  // (chg came back from a swap with the snapshot)
    }
    share_update(c);  // the interval just sampled: shared time counted up to now
    if (rc >= 0) {
      const int64_t dt = mono_ns() - s0;
      c->hwc_dt_ewma = c->hwc_dt_ewma > 0 ? 0.875 * c->hwc_dt_ewma + 0.125 * (double)dt : (double)dt;
      std::lock_guard<std::mutex> g(c->snap_mu);
      c->snap_blk = blk;
      c->snap_se.swap(se);
      c->snap_x.swap(xs);
      c->snap_own.swap(own);
      c->snap_chg.swap(chg);
      c->snap_t = s0;
      c->snap_share = c->share_ns;
      c->snap_seq++;
      c->hwc_ns += dt;
      if (dt > c->hwc_ns_max) c->hwc_ns_max = dt;
      c->hwc_samples++;
      c->hwc_period_sum_ns += last_hw ? s0 - last_hw : (int64_t)c->hwc_period_us * 1000;
      if (sw_since_hw && last_hw) {  // an interval the table changed in: the time-shared cadence
        c->ts_gap_sum += s0 - last_hw;
        c->ts_gaps++;
      }
      if (burst) c->hwc_burst_samples++;
      if (slow) c->hwc_slow_samples.fetch_add(1, std::memory_order_relaxed);
    }
    sw_since_hw = false;
    last_hw = s0;
    (void)t0;
    return rc >= 0;
  };
  while (!c->hwc_stop.load(std::memory_order_acquire)) {
    const int64_t t0 = mono_ns();
    const int64_t tick = (int64_t)c->hwc_period_us * 1000;
    const bool on_tick = t0 >= next_tick;
    bool sampled = false;
    if (on_tick) {
      next_tick = t0 + tick;
      // 1. watch: the modeled block (every tick with the watch on, else only
      //    with a hardware sample)
      const uint64_t sw = c->flushes.load(std::memory_order_relaxed);  // table publishes that changed an owner
      if (c->hwc_watch || sw != last_sw || t0 < burst_until || t0 - last_hw >= c->hwc_next_period_ns - tick / 4) {
        if (!read_block(c, blk.data())) break;
      }
      bool trig = false;
      for (int t = 0; t < kMaxTenants; ++t) {
        u64 di = 0, dm = 0;
        for (int x = 0; x < kXcds; ++x) {
          const size_t i = ((size_t)t * kXcds + x) * kNumPmc;
          di += dpos(blk[i], watch_prev[i]);
          dm += dpos(blk[i + 3], watch_prev[i + 3]);
        }
        if (di < 1000000) continue;  // too little work in this tick to judge
        const double r = (double)(dm + 1) / (double)di;
        if (watch_primed && watch_rate[t] > 0 && (r > 3.0 * watch_rate[t] || r * 3.0 < watch_rate[t])) trig = true;
        watch_rate[t] = watch_rate[t] > 0 ? 0.5 * watch_rate[t] + 0.5 * r : r;
      }
      std::copy(blk.begin(), blk.end(), watch_prev.begin());
      watch_primed = true;
      if (sw != last_sw) last_change = t0;
      last_sw = sw;
      if (trig) {
        burst_until = t0 + (int64_t)c->hwc_burst_ms * 1000000;
        c->hwc_triggers.fetch_add(1, std::memory_order_relaxed);
      }
      if (c->hwc_budget_pct > 0) {  // refill the sample budget
        const double dt = c->hwc_dt_ewma > 0 ? c->hwc_dt_ewma : 150000.0;
        if (c->hwc_tok_ns) c->hwc_tokens += (double)(t0 - c->hwc_tok_ns) * c->hwc_budget_pct / 100.0 / dt;
        c->hwc_tokens = std::min(c->hwc_tokens, (double)c->hwc_bucket);
        c->hwc_tok_ns = t0;
      }
    }
    // 2. switch-aligned samples.  Per partition p: settled = its last change
    //    is a drain guard old; open = a sample fell inside its current
    //    tenure, at least a guard after the tenure began (the tenure has a
    //    window that its next switch closes).  A sample is taken
    //    * one guard after the FIRST change of an open partition (closes its
    //      window, however soon further changes follow);
    //    * when a changed partition settles into a long tenure (>= long_us
    //      left of its quantum, or a quantum the table's writer did not give:
    //      manual tables) -- opens its window at the start;
    //    * for short tenures, as a budgeted pair: when one settles, the bucket
    //      holds 3 tokens, and the pair gap has passed.
    int64_t wake_at = next_tick;
    u32 changed = 0, q[P];
    int64_t chg[P], first[P];
    {
      std::lock_guard<std::mutex> g(c->mu);
      changed = c->sw_changed;
      std::memcpy(chg, c->part_chg_ns, sizeof(chg));
      std::memcpy(first, c->sw_first_p, sizeof(first));
      std::memcpy(q, c->part_q_us, sizeof(q));
      seen_pub = c->sw_last_ns;
    }
    const int64_t guard = guard_ns(c);
    const int64_t long_ns = (int64_t)c->hwc_long_us * 1000;
    auto consume = [&](u32 bits) {
      std::lock_guard<std::mutex> g(c->mu);
      c->sw_changed &= ~bits;
    };
    if (changed) sw_since_hw = true;
    if (changed && !c->hwc_align) {
      consume(changed);
      open = 0;
    } else if (changed) {
      u32 settled = 0, lngb = 0;
      int64_t next_settle = INT64_MAX, close_due = INT64_MAX;
      for (int p = 0; p < P; ++p) {
        if (!((changed >> p) & 1u)) continue;
        if (t0 - chg[p] >= guard) {
          settled |= 1u << p;
          if (q[p] == 0 || chg[p] + (int64_t)q[p] * 1000 - t0 >= long_ns) lngb |= 1u << p;
        } else {
          next_settle = std::min(next_settle, chg[p] + guard);
        }
        if ((open >> p) & 1u) close_due = std::min(close_due, first[p] + guard);
      }
      const u32 close = changed & open;
      const bool want_close = close && t0 >= close_due;
      rng ^= rng << 13;
      rng ^= rng >> 7;
      rng ^= rng << 17;
      const bool budgeted = c->hwc_budget_pct > 0;
      const bool lng = lngb != 0;
      const bool shrt = settled && !lng && (!budgeted || c->hwc_tokens >= 3.0) && t0 >= next_pair;
      const bool want = want_close || lng || shrt;
      if (want && (!budgeted || c->hwc_tokens >= 1.0)) {
        burst = slow = false;
        sampled = sample(t0);
        c->align_samples++;
        if (want_close) c->align_close++;
        if (lng) c->align_long++;
        if (shrt) {
          c->align_short++;
          // the next pair a jittered pair_gap_us on: at most ~1/gap short windows,
          // landing on every co-sharer of a lockstep rotation in turn
          next_pair = t0 + (int64_t)c->hwc_pair_gap_us * 1000 * (3 + (int64_t)(rng % 3)) / 4;
        }
        open &= ~changed;  // every changed partition's previous tenure ended
        open |= lng ? lngb : (shrt ? settled : 0u);
        consume(settled);  // an unsettled change is decided once it settles
      } else {
        if (want) c->align_denied++;
        if (settled) {  // settled without a sample: no window for these tenures
          open &= ~settled;
          consume(settled);
        }
        if (close && !want_close) wake_at = std::min(wake_at, close_due);
      }
      if (next_settle != INT64_MAX) wake_at = std::min(wake_at, next_settle);
    }
    // 2b. a short window closes BEFORE its tenure's switch: one sample time
    //     plus a margin ahead of the end of the quantum its owner was given
    //     (after the switch, the drain guard and the sample itself would take
    //     a third of a 1 ms tenure); a switch that comes early closes it as above
    if (c->hwc_align && !sampled && open) {
      const int64_t lead = (int64_t)c->hwc_dt_ewma + 50000;
      u32 pre = 0;
      int64_t pre_due = INT64_MAX;
      for (int p = 0; p < P; ++p) {
        if (!((open >> p) & 1u) || ((changed >> p) & 1u) || q[p] == 0 || (int64_t)q[p] * 1000 >= long_ns) continue;
        const int64_t due = chg[p] + (int64_t)q[p] * 1000 - lead;
        if (t0 >= due)
          pre |= 1u << p;
        else
          pre_due = std::min(pre_due, due);
      }
      if (pre && (c->hwc_budget_pct <= 0 || c->hwc_tokens >= 1.0)) {
        burst = slow = false;
        sampled = sample(t0);
        c->align_samples++;
        c->align_close++;
        open &= ~pre;
      } else if (pre) {
        c->align_denied++;
        open &= ~pre;
      }
      if (pre_due != INT64_MAX) wake_at = std::min(wake_at, pre_due);
    }
    // 3. burst / background sample on a tick
    if (on_tick && !sampled) {
      slow = c->hwc_slow_us > c->hwc_period_us && t0 - last_change >= kSteadyNs;
      int64_t period = slow ? (int64_t)c->hwc_slow_us * 1000 : tick;
      if (c->hwc_duty_pct > 0) period = std::max(period, (int64_t)(c->hwc_dt_ewma * 100.0 / c->hwc_duty_pct));
      c->hwc_next_period_ns = period;
      const bool due = t0 - last_hw >= period - tick / 4;
      burst = t0 < burst_until && !due;
      if (burst && c->hwc_budget_pct > 0 && c->hwc_tokens < 1.0) {
        burst = false;
        c->hwc_denied++;
      }
      if (burst || due) {
        sample(t0);
        // a sample inside a settled long tenure opens its window (closed at its next switch)
        std::lock_guard<std::mutex> g(c->mu);
        for (int p = 0; p < P; ++p)
          if (!((c->sw_changed >> p) & 1u) && t0 - c->part_chg_ns[p] >= guard &&
              (c->part_q_us[p] == 0 || c->part_chg_ns[p] + (int64_t)c->part_q_us[p] * 1000 - t0 >= long_ns))
            open |= 1u << p;
      }
    }
    // 3b. measurement tenures for tenants with no clean window lately (no
    //     lock of ours held: the engine call takes the engine lock, whose
    //     holders take c->mu)
    if (on_tick && c->hwc_align && c->hwc_measure_ms > 0 && c->engine && !c->muxed) {
      const int64_t ms = (int64_t)c->hwc_measure_ms * 1000000;
      int64_t ran[kMaxTenants], cln[kMaxTenants];
      {
        std::lock_guard<std::mutex> g(c->snap_mu);
        std::memcpy(ran, c->last_ran_ns, sizeof(ran));
        std::memcpy(cln, c->last_clean_ns, sizeof(cln));
      }
      const uint32_t want = (uint32_t)(c->hwc_long_us + guard_ns(c) / 1000 + 2 * (int64_t)(c->hwc_dt_ewma / 1000) + 300);
      for (int t = 0; t < kMaxTenants; ++t)
        if (ran[t] && t0 - ran[t] < ms && t0 - cln[t] > ms && t0 - c->measure_req_ns[t] > ms) {
          c->measure_req_ns[t] = t0;
          if (gpbs_tenant_measure(c->engine, t, want) >= 0) c->measure_reqs++;
        }
    }
    // 4. sleep until the next tick, a pending switch sample, or a new publish
    std::unique_lock<std::mutex> lk(c->mu);
    c->cv.wait_until(lk, std::chrono::steady_clock::time_point(std::chrono::nanoseconds(wake_at)), [&] {
      return c->hwc_stop.load(std::memory_order_acquire) || (c->hwc_align && c->sw_last_ns != seen_pub);
    });
  }
}


// Fold one attribution result into the per-tenant totals and the pending
// metric deltas (snap_mu held).  `mod`: the same interval's modeled deltas,
// `pres`: each tenant's largest owned share of a partition over it, `t_s`:
// the interval's closing sample time.  Per tenant that ran:
//   clean     a clean window: its clean counts reach the PBS metric, and a
//             window that covers all its counts recalibrates hardware/model;
//   fallback  no clean window, substantial presence, the last clean window
//             older than hwc_stale_us and a calibration: modeled x ratio;
//   skipped   no clean window, substantial presence, otherwise: nothing;
//   sliver    owned < (100 - clean_pct) % of the interval: nothing.
void hwc_fold(GpuCtx* c, const HwcAttrOut& o, const double (*mod)[kNumPmc], const double* pres, int64_t t_s) {
  if (!o.valid) return;
  const double sub = c->clean_pct > 0 ? (100.0 - c->clean_pct) / 100.0 : 0.0;
  for (int t = 0; t < kMaxTenants; ++t) {
    for (int k = 0; k < kNumPmc; ++k)
      if (o.add[t][k] > 0) c->att_total[t][k] += o.add[t][k];
    if (o.add[t][0] <= 0) continue;  // did not run in the interval
    c->last_ran_ns[t] = t_s;
    const bool clean = c->clean_pct <= 0 || o.addc[t][0] > 0;
    // 1 ms cadence: a calibrated tenant reported this interval tick by tick
    // from its calibrated model (cadence_tick); its hardware windows only
    // re-anchor the calibration
    const bool ticked = c->model_cadence && c->cnt_bar && c->cal[t][0] > 0;
    double m[kNumPmc] = {0, 0, 0, 0};
    if (clean) {
      c->clean_periods++;
      c->t_clean[t]++;
      c->last_clean_ns[t] = t_s;
      for (int k = 0; k < kNumPmc; ++k) m[k] = c->clean_pct > 0 ? o.addc[t][k] : o.add[t][k];
      // the window holds (nearly) all the tenant ran: hardware over modeled
      if (mod && mod[t][0] > 0 && o.addc[t][0] >= 0.9 * o.add[t][0])
        for (int k = 0; k < kNumPmc; ++k)
          if (mod[t][k] > 0 && o.add[t][k] > 0) {
            const double r = o.add[t][k] / mod[t][k];
            c->cal[t][k] = c->cal[t][k] > 0 ? 0.75 * c->cal[t][k] + 0.25 * r : r;
          }
      if (ticked) continue;
    } else if (pres && pres[t] < sub) {
      c->sliver_periods++;
      c->t_sliver[t]++;
      continue;
    } else if (ticked) {
      continue;
    } else {
      const bool stale = t_s - c->last_clean_ns[t] > (int64_t)c->hwc_stale_us * 1000;
      if (c->model_fallback && stale && mod && mod[t][0] > 0 && c->cal[t][0] > 0) {
        c->fallback_periods++;
        c->t_fallback[t]++;
        for (int k = 0; k < kNumPmc; ++k) m[k] = mod[t][k] * c->cal[t][k];
      } else {
        c->skipped_periods++;
        c->t_skipped[t]++;
        continue;
      }
    }
    for (int k = 0; k < kNumPmc; ++k)
      if (m[k] > 0) {
        c->last_delta[t][k] += (u64)(m[k] + 0.5);
        c->metric_sum[k] += m[k];
        c->met_total[t][k] += m[k];
      }
  }
  for (int k = 0; k < kNumPmc; ++k) {
    c->hw_sum[k] += o.hw_sum[k];
    c->unatt[k] += o.unatt[k];
  }
}

// The newest snapshot as attribution input (snap_mu held).
void hwc_fill_in(GpuCtx* c, HwcAttrIn& in) {
  std::memcpy(in.se_cur, c->snap_se.data(), sizeof(in.se_cur));
  std::memcpy(in.x_cur, c->snap_x.data(), sizeof(in.x_cur));
  std::memcpy(in.own_cur, c->snap_own.data(), sizeof(in.own_cur));
  for (int k = 0; k < kNumPmc; ++k) in.slot_se[k] = (u32)c->slot_se[k];
  in.se_mode = (u32)__atomic_load_n(&c->se_mode, __ATOMIC_ACQUIRE);
  in.clean_pct = (u32)c->clean_pct;
  in.shared = c->snap_share > c->share_prev;
  in.prime = !c->hw_primed;
  u32 hi = 0;  // tenants that ever owned a partition (owned time only grows)
  for (int t = kMaxTenants - 1; t >= 0 && !hi; --t)
    for (int x = 0; x < kAttrP; ++x)
      if (in.own_cur[t * kAttrP + x]) {
        hi = (u32)t + 1;
        break;
      }
  in.nt_hi = hi ? hi : 1;
  // drain guard: the interval opens at the last consumed sample; a partition
  // whose last owner change came at least a guard before it starts clean --
  // in an interval of at least three guards, so a drain that outlasts the
  // guard stays a small part of the window
  // (and no owner change in the interval's head: hwc_drained_bits)
  u32 dr = 0;
  if (c->used_chg.size() == (size_t)kAttrP && c->snap_chg.size() == (size_t)kAttrP)
    dr = hwc_drained_bits(c->used_t, c->snap_t, c->used_chg.data(), c->snap_chg.data(), guard_ns(c),
                          (u32)c->clean_pct);
  in.drained = dr;
}

// Modeled per-tile counters over the same interval (cross-check and
// calibrated fallback), and each tenant's largest owned share of a
// partition over it (host).
void hwc_model(GpuCtx* c) {
  std::memset(c->mod_cur, 0, sizeof(c->mod_cur));
  std::memset(c->pres_cur, 0, sizeof(c->pres_cur));
  if (!c->hw_primed) return;
  for (int t = 0; t < kMaxTenants; ++t)
    for (int k = 0; k < kNumPmc; ++k) {
      double md = 0;
      for (int x = 0; x < kXcds; ++x) {
        const size_t i = ((size_t)t * kXcds + x) * kNumPmc + k;
        md += (double)dpos(c->snap_blk[i], c->blk_prev[i]);
      }
      c->mod_cur[t][k] = md;
      c->mod_total[t][k] += md;
      c->model_sum[k] += md;
    }
  if (c->own_prev.size() != c->snap_own.size()) return;
  double span = 0;
  static thread_local double tot[kAttrP];
  for (int p = 0; p < kAttrP; ++p) {
    tot[p] = 0;
    for (int t = 0; t < kMaxTenants; ++t) {
      const int64_t d = c->snap_own[(size_t)t * kAttrP + p] - c->own_prev[(size_t)t * kAttrP + p];
      if (d > 0) tot[p] += (double)d;
    }
    span = std::max(span, tot[p]);
  }
  if (span <= 0) return;
  for (int t = 0; t < kMaxTenants; ++t)
    for (int p = 0; p < kAttrP; ++p) {
      const int64_t d = c->snap_own[(size_t)t * kAttrP + p] - c->own_prev[(size_t)t * kAttrP + p];
      if (d > 0) c->pres_cur[t] = std::max(c->pres_cur[t], (double)d / span);
    }
}

// Consume the newest sampler snapshot (snap_mu held).  Device path: harvest
// the attribution launched at the previous call if it has finished, then
// launch one for the newest snapshot; a launch still running (a tail) makes
// this call launch nothing, and the next one covers both intervals.  With
// `wait`, block until this call's launch is harvested (tools, not under the
// engine lock).  Returns 1 if a snapshot was consumed.
int hwc_consume(GpuCtx* c, bool wait) {
  if (c->dev_attr && c->attr_pending) {
    const hipError_t q = wait ? hipEventSynchronize(c->attr_ev) : hipEventQuery(c->attr_ev);
    if (q == hipSuccess) {
      hwc_fold(c, *c->h_aout, c->mod_inflight, c->pres_inflight, c->t_inflight);
      c->attr_pending = false;
      const uint64_t tk = (uint32_t)(c->h_aout->pad[1] - c->h_aout->pad[0]);
      c->attr_harvested++;
      c->attr_ticks_sum += tk;
      c->attr_ticks_max = std::max(c->attr_ticks_max, tk);
      c->attr_lag_sum_ns += mono_ns() - c->attr_launch_ns;
    } else {
      c->attr_busy_skips++;
      return 0;
    }
  }
  if (c->snap_seq == c->used_seq || c->snap_own.empty()) return 0;
  c->used_seq = c->snap_seq;
  hwc_model(c);
  bool done = false;
  if (c->dev_attr) {
    hwc_fill_in(c, *c->h_ain);
    // the snapshot reaches the kernel through the BAR (host streaming
    // stores into fine-grained VRAM): round 5's staging hipMemcpyAsync ran
    // as a copyBuffer blit kernel on the tenants' CUs at every sample
    if (c->f_ain) bar_store(c->f_ain, c->h_ain, hwc_attr_in_bytes(*c->h_ain));
    if (gpbs_hip_hwc_attribute2(c->h_ain, c->f_ain ? c->f_ain : c->d_ain, c->d_ast, c->h_aout, c->sched_stream,
                                c->f_ain ? 0 : 1) == 0 &&
        hipEventRecord(c->attr_ev, c->sched_stream) == hipSuccess) {
      c->attr_pending = true;
      c->attr_launches++;
      c->attr_launch_ns = mono_ns();
      std::memcpy(c->mod_inflight, c->mod_cur, sizeof(c->mod_cur));
      std::memcpy(c->pres_inflight, c->pres_cur, sizeof(c->pres_cur));
      c->t_inflight = c->snap_t;
      done = true;
      if (wait && hipEventSynchronize(c->attr_ev) == hipSuccess) {
        hwc_fold(c, *c->h_aout, c->mod_inflight, c->pres_inflight, c->t_inflight);
        c->attr_pending = false;
      }
    }
  }
  if (!done) {  // host path (param device_attr 0, or a failed launch)
    static thread_local HwcAttrIn in;
    static thread_local HwcAttrOut out;
    hwc_fill_in(c, in);
    hwc_attr_host(in, c->hst, out);
    hwc_fold(c, out, c->mod_cur, c->pres_cur, c->snap_t);
    c->attr_host++;
  }
  c->blk_prev = c->snap_blk;
  c->own_prev = c->snap_own;
  c->used_chg = c->snap_chg;
  c->used_t = c->snap_t;
  c->share_prev = c->snap_share;
  c->hw_primed = true;
  return 1;
}

// One metric tick of the 1 ms cadence (snap_mu held): every calibrated
// tenant's modeled deltas since the previous tick, scaled per counter by its
// hardware/model ratio, go to its pending metric deltas.  The block is read
// through the BAR (no GPU work); without a host-readable block the cadence
// is off and the hardware windows report, as before.
void cadence_tick(GpuCtx* c) {
  constexpr int kRow = kXcds * kNumPmc;
  if (!c->model_cadence || !c->cnt_bar) return;
  const int rows = std::min(kMaxTenants, std::max(1, c->cnt_rows.load(std::memory_order_relaxed)));
  static thread_local std::vector<u64> cur;
  cur.assign((size_t)kMaxTenants * kRow, 0);
  bar_read(c->d_cnt, cur.data(), sizeof(u64) * (size_t)rows * kRow);
  if (!c->cad_primed || c->cad_prev.size() != cur.size()) {
    c->cad_prev = cur;
    c->cad_primed = true;
    return;
  }
  {
    int64_t* d = c->cad_dbg[c->cad_calls % 512];
    d[0] = mono_ns();
    for (int tt = 1; tt <= 2 && tt < rows; ++tt) {
      u64 v = 0;
      for (int x = 0; x < kXcds; ++x) v += cur[((size_t)tt * kXcds + x) * kNumPmc];
      d[tt] = (int64_t)v;
    }
  }
  c->cad_calls++;
  for (int t = 0; t < rows; ++t) {
    double md[kNumPmc] = {0, 0, 0, 0};
    for (int x = 0; x < kXcds; ++x)
      for (int k = 0; k < kNumPmc; ++k) {
        const size_t i = ((size_t)t * kXcds + x) * kNumPmc + k;
        md[k] += (double)dpos(cur[i], c->cad_prev[i]);
      }
    if (md[0] <= 0) continue;
    c->t_moved[t]++;
    if (c->cal[t][0] <= 0) continue;
    for (int k = 0; k < kNumPmc; ++k) {
      const double v = md[k] * c->cal[t][k];
      if (v <= 0) continue;
      c->last_delta[t][k] += (u64)(v + 0.5);
      c->metric_sum[k] += v;
      c->met_total[t][k] += v;
    }
    c->t_model[t]++;
  }
  c->cad_prev.swap(cur);
}

int hwc_tenant_deltas(GpuCtx* c, int n, const int* tenants, uint64_t* out) {
  const int64_t t0 = mono_ns();
  RoctxRange rr("gpbs:metric_tick");
  {
    std::lock_guard<std::mutex> g(c->snap_mu);
    hwc_consume(c, false);
    cadence_tick(c);
    for (int k = 0; k < n; ++k) {  // per-tenant metric cadence: periods that delivered anything
      const int t = tenants[k];
      if (t < 0 || t >= kMaxTenants || !c->last_delta[t][0]) continue;
      if (!c->t_delivered[t]++) c->t_first_ns[t] = t0;
      c->t_last_ns[t] = t0;
    }
  }
  // No new snapshot since the previous tick: every tenant reads zero
  // instructions and the PBS idle-sample rule (Q14) skips the period.
  for (int k = 0; k < n; ++k)
    for (int i = 0; i < kNumPmc; ++i) {
      const int t = tenants[k];
      out[k * kNumPmc + i] = (t >= 0 && t < kMaxTenants) ? c->last_delta[t][i] : 0;
      if (t >= 0 && t < kMaxTenants) c->last_delta[t][i] = 0;
    }
  c->metric_calls++;
  c->metric_ns += mono_ns() - t0;
  return 0;
}

// The runners' measured switch costs (drain + ramp) to the engine, where they
// floor each tenant's quantum in a time-shared region (boot switch_floor_x).
// Under the engine lock (the metric tick; the mutex is recursive), pushed when
// a tenant's cost moved by more than 5 %.
void push_switch_costs(GpuCtx* c, int n, const int* tenants) {
  for (int k = 0; k < n; ++k) {
    const int t = tenants[k];
    if (t < 0 || t >= kMaxTenants) continue;
    const uint64_t nd = c->swc_drain_n[t].load(std::memory_order_relaxed);
    const uint64_t nr = c->swc_ramp_n[t].load(std::memory_order_relaxed);
    if (!nd && !nr) continue;
    const int64_t cost = (nd ? c->swc_drain_ns[t].load(std::memory_order_relaxed) : 0) +
                         (nr ? c->swc_ramp_ns[t].load(std::memory_order_relaxed) : 0);
    const int64_t last = c->swc_pushed_ns[t];
    if (last && std::llabs(cost - last) * 20 < last) continue;
    c->swc_pushed_ns[t] = cost;
    gpbs_tenant_switch_cost(c->engine, t, (uint64_t)std::max<int64_t>(cost, 0));
  }
}

int ctr_tenant_deltas(void* user, int n, const int* tenants, uint64_t* out) {
  GpuCtx* c = (GpuCtx*)user;
  if (n > kMaxTenants) return -22;
  if (c->engine) {  // engine lock held: refresh the class cache launch() reads
    for (int k = 0; k < n; ++k)
      if (tenants[k] >= 0 && tenants[k] < kMaxTenants)
        c->cls_cache[tenants[k]].store(gpbs_tenant_class(c->engine, tenants[k]), std::memory_order_relaxed);
    push_switch_costs(c, n, tenants);
  }
  if (c->hwc) return hwc_tenant_deltas(c, n, tenants, out);
  const int64_t t0 = mono_ns();
  RoctxRange rr("gpbs:metric_tick");
  if (c->cnt_bar) {
    // Modeled counters only (no live sampler): the block crosses the BAR and
    // is reduced here -- no k_counter_reduce on the tenants' queues (a
    // rocprofv3 kernel trace of --counters model showed it at 1 kHz,
    // profiles/r6/s45_rocprof_summary.txt)
    static thread_local std::vector<u64> blk;
    blk.resize((size_t)kMaxTenants * kXcds * kNumPmc);
    read_block(c, blk.data());
    const int rows = std::min(kMaxTenants, std::max(1, c->cnt_rows.load(std::memory_order_relaxed)));
    for (int k = 0; k < n; ++k) {
      const int t = tenants[k];
      for (int i = 0; i < kNumPmc; ++i) out[k * kNumPmc + i] = 0;
      if (t < 0 || t >= rows) continue;
      for (int x = 0; x < kXcds; ++x)
        for (int i = 0; i < kNumPmc; ++i) {
          const size_t j = ((size_t)t * kXcds + x) * kNumPmc + i;
          out[k * kNumPmc + i] += dpos(blk[j], c->red_prev[j]);  // Q5
          c->red_prev[j] = blk[j];
        }
    }
    c->metric_calls++;
    c->metric_ns += mono_ns() - t0;
    return 0;
  }
  if (c->red_pending && hipEventQuery(c->red_ev) == hipErrorNotReady) {
    // The previous reduce has not finished (a tail, ~0.1 % of periods): never
    // wait for it under the engine lock.  This period reports nothing (the
    // idle-sample rule skips it) and the next tick harvests both periods.
    for (int k = 0; k < n * kNumPmc; ++k) out[k] = 0;
    c->metric_calls++;
    c->metric_ns += mono_ns() - t0;
    return 0;
  }
  if (c->red_pending) {
    const int* ids = c->red_buf ? c->h_ids2 : c->h_ids;
    const u64* res = c->red_buf ? c->h_out2 : c->h_out;
    for (int k = 0; k < c->red_n; ++k)
      if (ids[k] >= 0 && ids[k] < kMaxTenants)
        for (int i = 0; i < kNumPmc; ++i) c->last_delta[ids[k]][i] += res[k * kNumPmc + i];
    c->red_pending = false;
  }
  for (int k = 0; k < n; ++k)
    for (int i = 0; i < kNumPmc; ++i) {
      const int t = tenants[k];
      out[k * kNumPmc + i] = (t >= 0 && t < kMaxTenants) ? c->last_delta[t][i] : 0;
      if (t >= 0 && t < kMaxTenants) c->last_delta[t][i] = 0;
    }
  c->red_buf ^= 1;
  int* ids = c->red_buf ? c->h_ids2 : c->h_ids;
  u64* res = c->red_buf ? c->h_out2 : c->h_out;
  for (int i = 0; i < n; ++i) ids[i] = tenants[i] < kMaxTenants ? tenants[i] : -1;
  if (gpbs_hip_counter_reduce(c->d_cnt, c->d_prev, ids, n, res, c->sched_stream)) return -5;
  hipEventRecord(c->red_ev, c->sched_stream);
  c->red_pending = true;
  c->red_n = n;
  c->metric_calls++;
  c->metric_ns += mono_ns() - t0;
  return 0;
}

constexpr int64_t kAdaptPollNs = 200000;  // 0.2 ms of the 1 ms metric period

int ctr_adapt_batch(void* user, int n, const int*, const uint64_t* deltas, const uint64_t* ssum, const uint64_t* scnt,
                    gpbs_adapt_state_t* states, const gpbs_adapt_params_t* p) {
  GpuCtx* c = (GpuCtx*)user;
  if (n > kMaxTenants) return -22;
  const int64_t t0 = mono_ns();
  RoctxRange rr("gpbs:adapt_device");
  // The engine lock is held here: never block on the device.  A previous
  // launch still running (its buffers are in use) or a result not back
  // within the poll budget makes this period fall back to the host
  // adapt_update (bit-identical), and the late result is discarded.
  c->adapt_calls++;
  if (c->adapt_pending) {
    if (hipEventQuery(c->adapt_ev) == hipErrorNotReady) {
      c->adapt_busy++;
      return -11;
    }
    c->adapt_pending = false;
  }
  std::memcpy(c->h_states, states, sizeof(gpbs_adapt_state_t) * n);
  std::memcpy(c->h_adelta, deltas, sizeof(u64) * 4 * n);
  std::memcpy(c->h_spin, ssum, sizeof(u64) * n);
  std::memcpy(c->h_spin + kMaxTenants, scnt, sizeof(u64) * n);
  if (gpbs_hip_adapt(c->h_states, c->h_adelta, c->h_spin, c->h_spin + kMaxTenants, n, p, c->h_dirs, c->sched_stream))
    return -5;
  hipEventRecord(c->adapt_ev, c->sched_stream);
  c->adapt_pending = true;
  for (;;) {
    const hipError_t q = hipEventQuery(c->adapt_ev);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) return -5;
    if (mono_ns() - t0 > kAdaptPollNs) {
      c->adapt_late++;
      c->metric_ns += mono_ns() - t0;
      return -11;
    }
  }
  c->adapt_pending = false;
  std::memcpy(states, c->h_states, sizeof(gpbs_adapt_state_t) * n);
  c->metric_ns += mono_ns() - t0;
  return 0;
}

int ctr_adapt_launch(void* user, int n, const int* tenants, const uint64_t* deltas, const uint64_t* ssum,
                     const uint64_t* scnt, const gpbs_adapt_state_t* states, const gpbs_adapt_params_t* p) {
  GpuCtx* c = (GpuCtx*)user;
  if (n <= 0 || n > kMaxTenants) return -22;
  RoctxRange rr("gpbs:adapt_launch");
  int b = -1;
  for (int i = 0; i < GpuCtx::kAbuf; ++i) {
    GpuCtx::AdaptBuf& B = c->abuf[i];
    // a dropped result that landed, or an orphan nobody harvested: free once
    // the kernel is done
    const bool orphan = B.state == 1 && c->async_launches - B.gen > GpuCtx::kAbufOrphan;
    if ((B.state == 2 || orphan) && hipEventQuery(B.ev) == hipSuccess) B.state = 0;
    // the caller's own previous launch is superseded by this one (it did not
    // harvest it: its tick recomputed that period on the host)
    if (B.state == 1 && B.n == n && std::memcmp(B.ids, tenants, sizeof(int) * n) == 0) B.state = 2;
    if (B.state == 0 && b < 0) b = i;
  }
  if (b < 0) {
    c->async_busy++;
    return -11;
  }
  GpuCtx::AdaptBuf& B = c->abuf[b];
  std::memcpy(B.st, states, sizeof(gpbs_adapt_state_t) * n);
  std::memcpy(B.delta, deltas, sizeof(u64) * 4 * n);
  std::memcpy(B.spin, ssum, sizeof(u64) * n);
  std::memcpy(B.spin + kMaxTenants, scnt, sizeof(u64) * n);
  std::memcpy(B.ids, tenants, sizeof(int) * n);
  B.n = n;
  if (gpbs_hip_adapt(B.st, B.delta, B.spin, B.spin + kMaxTenants, n, p, nullptr, c->sched_stream) ||
      hipEventRecord(B.ev, c->sched_stream) != hipSuccess)
    return -5;
  B.state = 1;
  B.gen = ++c->async_launches;
  return 0;
}

// tenants_out holds, on entry, the ids the caller launched (max of them):
// harvest that launch and no other pool's.
int ctr_adapt_harvest(void* user, int max, int* tenants_out, gpbs_adapt_state_t* states_out) {
  GpuCtx* c = (GpuCtx*)user;
  if (max <= 0 || max > kMaxTenants || !tenants_out) return -22;
  GpuCtx::AdaptBuf* B = nullptr;
  for (auto& X : c->abuf)
    if (X.state == 1 && X.n == max && std::memcmp(X.ids, tenants_out, sizeof(int) * max) == 0 &&
        (!B || X.gen > B->gen))
      B = &X;
  if (!B) return -22;
  if (hipEventQuery(B->ev) != hipSuccess) {
    B->state = 2;  // the engine recomputes this period on the host; drop the result when it lands
    c->async_late++;
    return -11;
  }
  std::memcpy(states_out, B->st, sizeof(gpbs_adapt_state_t) * max);
  std::memcpy(tenants_out, B->ids, sizeof(int) * max);
  B->state = 0;
  return max;
}

// --------------------------------------------------------------------- runner

enum Kind { K_GEMM = 1, K_STREAM = 2, K_REDUCE = 3, K_GEMV = 4, K_ALLREDUCE = 5 };

// ---- all-reduce tenant over IPC-mapped peer buffers (coll_kernels.hip) ----
// Host mirror of the device CollDesc: per rank its input, output and flag
// words as mapped into this process (own buffers for our rank, IPC-opened
// peers for the others).
constexpr int kCollMax = 8;
struct CollDescHost {
  const void* in[kCollMax];
  void* out[kCollMax];
  u32* flags[kCollMax];
  u32 rank, world;
  u64 n8;
};

struct Coll {
  int device = 0, rank = 0, world = 1;
  size_t bytes = 0;
  void* in = nullptr;
  void* out = nullptr;
  u32* flags = nullptr;
  void* peer[3][kCollMax] = {};  // opened IPC mappings: in, out, flags
  CollDescHost desc{};
  void* d_desc = nullptr;
};

}  // namespace

extern "C" {

typedef struct gpbs_runner_cfg {
  int kind;
  int tenant;       // engine tenant id (< 64); also the kernel's owner id
  int gate;         // 1: obey the partition table; 0: run anywhere (policy "none")
  int priority;     // stream priority: 0 normal, 1 high
  int depth;        // units in flight
  int grid;         // 0 = default persistent grid
  int M, N, K;      // GEMM / GEMV shapes
  int chunk_bytes;  // stream / reduce chunk
  int engine_wake;  // 1: wake/block engine slots as work arrives/drains
  int reserved;
  unsigned long long bytes;  // stream / reduce bytes
  void *a, *b, *c;           // device buffers (caller-owned)
  // Alternate workload (phase-changing tenant): a second kind with its own
  // shape and buffers; gpbs_runner_set_phase(r, 1) makes every FRESH unit use
  // it (a revoked unit resumes with the kind it started with).  alt_kind 0:
  // none.
  int alt_kind;
  int alt_M, alt_N, alt_K;
  int alt_chunk_bytes;
  int alt_reserved;
  unsigned long long alt_bytes;
  void *alt_a, *alt_b, *alt_c;
} gpbs_runner_cfg_t;

typedef struct gpbs_runner_stats {
  uint64_t units_done, launches, relaunches, waits_owner, submitted;
  int64_t busy_ns, wait_owner_ns, first_start_ns, last_done_ns;
  int64_t lat_sum_ns, lat_max_ns;
  uint64_t lat_count;
  uint64_t units_alt;  // of units_done: units of the alternate workload
  // revocation drain: from the table publish that took a partition from this
  // tenant to the end of the unit it interrupted (the unit's grid has left
  // every SE; until then the new owner's workgroups queue behind it)
  int64_t drain_sum_ns, drain_max_ns;
  uint64_t drain_count;
} gpbs_runner_stats_t;

}

namespace {

// Process-wide pool of CU-masked streams.  Every CU-masked stream is a
// hardware queue of its own and the process never gets one back; past the
// hardware scheduler's queue slots it oversubscribes and time-slices ALL
// queues, idle ones included.  Measured (scripts/queue_budget.py,
// profiles/r4/queue_budget*.log): a solo GEMM keeps its rate up to 20 extra
// masked queues and loses 24 % at 24, 63 % at 48; with the device-counting
// context running the knee moves down by about four queues.  So queues are
// pooled (a runner returns its queue when it closes or changes layout) and
// SHARED by key: runners that hold the same set of (XCD, SE) partitions --
// co-sharers of a time-shared region, which never run at the same time --
// launch on one queue.  Runners on different sets run concurrently and get
// their own queue: two of them on one queue run their units one after
// another (round 4 capped keyed queues at two per mask, and the 8mix split
// layouts -- three or four concurrent layouts per class half -- collapsed
// from 1.10 to 0.78 solo-equivalents).  Only past kMaskedBudget live queues
// on a device does a new layout share another key's least-held queue, and
// every such share is counted (cross_key_shares, reported with the run).
// The policy is host-only code (MaskedPoolCore), checked on the CPU by
// gpbs_hip_masked_pool_selftest with fake queue handles.
// Budget 10: the most layouts any mix runs at once is 8 (the 8mix static
// split: 3 compute blocks, 4 memory blocks, the latency lane); every created
// queue stays with the process, and past ~24 hardware queues in all (these,
// the 12 plain-stream queues, the profiler's) the hardware scheduler
// time-slices every queue: a full bench process that had created 16 ran its
// 8mix at 0.84-0.97 instead of 1.26-1.28 (profiles/r5/bench_s6_queue_growth.txt).
constexpr int kMaskedBudget = 10;
constexpr int kPipeCreateCap = 8;  // creating a queue only for a better pipe stops here
// Hardware queues land on the command processor's pipes round-robin in
// creation order (4 pipes): CU-masked queues whose creation indexes differ by
// a multiple of 4 share a pipe, and a GEMM dispatch waiting there for CUs
// holds up the other queue's dispatches -- a stream copy on the other half
// of the GPU keeps 0.61-0.64 of its rate next to back-to-back GEMMs on a
// same-pipe queue, 0.88-0.89 on any other (scripts/pipe_probe.py,
// profiles/r5/pipe_probe.txt).  That was the round-4 "bimodal 8mix" (slow
// runs had the GEMMs' queue and a stream's 4 pool indexes apart).  So a
// layout takes the queue whose pipe is least shared with the layouts running
// now -- another class half's queue costs 10, same half 1.
// The pipe is the index in the PROCESS's queue creation order, which also
// counts the plain-stream queues HIP creates lazily and the profiler's: a
// pool index mod 4 predicted nothing in a full bench process (s8: slow 8mix
// runs had the GEMMs on pool queue 6 and the streams on 5, 7 or 8).  So the
// pool creates all its queues in ONE burst at first use, nothing else
// creating queues in between (prealloc, under the pool lock), in the plan
// kPlan -- compute half on burst indexes 0, 4, 8 (one pipe), memory half on
// the other three pipes -- and only the relative pipes within the burst are
// used.  Round 4's preallocation (C M M C M) put a memory queue on the
// compute pipe, which is why it measured no better.
constexpr int kPipes = 4;
constexpr int kPlanLen = kMaskedBudget;
constexpr int kPlan[kPlanLen] = {0, 1, 1, 1, 0, 1, 1, 1, 0, 1};  // class half per burst index

struct MaskedPoolCore {
  struct Ent {
    int device;
    uint32_t m[8];
    hipStream_t s;
    uint32_t key;
    int refs;
    int pipe;  // creation index mod kPipes (in the device's burst)
    double load = 0;  // its holders' dispatch rates (launches / s, as they acquired it)
  };
  std::mutex mu;
  std::vector<Ent> ents;
  uint64_t created = 0, cross_key_shares = 0, pipe_shared_other = 0;
  int held_max = 0;  // high-water mark of queues held at once (reset with reset_max)
  int dev_created[16] = {};
  bool dev_burst[16] = {};

  // Create the device's queues in one burst: plan[i] picks masks[plan[i]]
  // for burst index i (pipe i mod kPipes).  Once per device; later creations
  // (an exclusive acquire with no idle queue) continue the count.
  template <class Create>
  int prealloc(int dev, const uint32_t* const masks[2], const int* plan, int n, Create&& create) {
    std::lock_guard<std::mutex> g(mu);
    const int dv = dev >= 0 && dev < 16 ? dev : 0;
    if (dev_burst[dv]) return 0;
    dev_burst[dv] = true;
    int made = 0;
    for (auto& e : ents) made += e.device == dev;
    if (made) return 0;  // queues exist already: their pipes are unknown, keep the incremental policy
    for (int i = 0; i < n; ++i) {
      hipStream_t s = create(masks[plan[i]]);
      if (!s) return -1;
      ents.push_back({dev, {}, s, 0, 0, i % kPipes});
      std::memcpy(ents.back().m, masks[plan[i]], sizeof(ents.back().m));
      created++;
      dev_created[dv]++;
    }
    return n;
  }

  int held_locked(int dev) const {
    int n = 0;
    for (const auto& e : ents) n += e.device == dev && e.refs > 0;
    return n;
  }
  // cost of running a layout of mask m / key k on `pipe` next to the held
  // queues: 10 per queue of the other class half (its dispatch waiting for
  // CUs holds this pipe), 1 per queue of the same half -- each weighted by
  // how busy that queue keeps the pipe (1 + its holders' launches per ms), so
  // a launch-bound tenant shares its pipe with the latency tenant's idle
  // queue rather than with a stream (slo mix: the MALL-sized tenant kept 0.284
  // of its solo rate on a pipe of its own or next to the latency queue, 0.200
  // next to a stream's queue, profiles/r6/s30)
  double pipe_cost(int dev, int pipe, const uint32_t m[8], uint32_t key, const Ent* self) const {
    double cost = 0;
    for (const auto& e : ents)
      if (&e != self && e.device == dev && e.refs > 0 && e.pipe == pipe && (key == 0 || e.key != key))
        cost += (std::memcmp(e.m, m, sizeof(e.m)) != 0 ? 10.0 : 1.0) * (1.0 + e.load / 1000.0);
    return cost;
  }
  // key 0: exclusive (never shared).  create(m) makes a new queue (nullptr on
  // failure).  Caller does not hold mu.
  template <class Create>
  hipStream_t acquire(int dev, const uint32_t m[8], uint32_t key, Create&& create, double load = 0) {
    std::lock_guard<std::mutex> g(mu);
    Ent* same = nullptr;   // this layout's queue
    Ent* idle = nullptr;   // the cheapest queue of this mask nobody holds
    Ent* least = nullptr;  // least-held keyed queue of this mask
    int live = 0;
    double idle_cost = 1e30;
    for (auto& e : ents) {
      if (e.device != dev) continue;
      live++;
      if (std::memcmp(e.m, m, sizeof(e.m)) != 0) continue;
      if (key && e.key == key && e.refs > 0 && (!same || e.refs < same->refs)) same = &e;
      if (e.refs == 0) {
        const double cst = pipe_cost(dev, e.pipe, m, key, &e) * 2 + (key && e.key == key ? 0 : 1);
        if (cst < idle_cost) idle = &e, idle_cost = cst;
      }
      if (e.key && e.refs > 0 && (!least || e.refs < least->refs)) least = &e;
    }
    const int dv = dev >= 0 && dev < 16 ? dev : 0;
    const int new_pipe = dev_created[dv] % kPipes;
    const double new_cost = pipe_cost(dev, new_pipe, m, key, nullptr) * 2 + 1;
    hipStream_t s = nullptr;
    Ent* got = nullptr;
    if (same) {
      same->refs++;
      got = same;
    } else if (idle && (idle_cost <= new_cost || live >= kPipeCreateCap)) {
      idle->key = key;
      idle->refs = 1;
      got = idle;
    } else if (live < kMaskedBudget || !key || !least) {
      s = create(m);
      if (!s) return nullptr;
      ents.push_back({dev, {}, s, key, 1, new_pipe});
      std::memcpy(ents.back().m, m, sizeof(ents.back().m));
      created++;
      dev_created[dv]++;
      got = &ents.back();
    } else {  // over budget: share another layout's queue (serialises the two)
      least->refs++;
      cross_key_shares++;
      got = least;
    }
    if (got != same && pipe_cost(dev, got->pipe, m, key, got) >= 10) pipe_shared_other++;
    got->load += load;
    held_max = std::max(held_max, held_locked(dev));
    return got->s;
  }
  void release(hipStream_t s, double load = 0) {
    if (!s) return;
    std::lock_guard<std::mutex> g(mu);
    for (auto& e : ents)
      if (e.s == s && e.refs > 0) {
        e.refs--;
        e.load = e.refs ? std::max(0.0, e.load - load) : 0.0;
        return;
      }
  }
  int pipe_of(hipStream_t s) {
    std::lock_guard<std::mutex> g(mu);
    for (auto& e : ents)
      if (e.s == s) return e.pipe;
    return -1;
  }
};
// The pool object is never destroyed (its streams must outlive any static
// teardown order); its queues are destroyed at exit, by an atexit handler
// registered after the HIP runtime came up -- so it runs before the runtime's
// own teardown and before a profiler's tool finalizer registered earlier.
// Left to the runtime's teardown, the CU-masked queues crashed every process
// run under rocprofv3 in __cxa_finalize after the tool had finalized
// (scripts/exit_probe.py: "pool" rc 139, "ctx0" without the pool rc 0).
void masked_pool_teardown();
MaskedPoolCore& masked_pool() {
  static MaskedPoolCore* p = [] {
    auto* q = new MaskedPoolCore;
    std::atexit(masked_pool_teardown);
    return q;
  }();
  return *p;
}
void masked_pool_teardown() {
  MaskedPoolCore& P = masked_pool();
  std::lock_guard<std::mutex> g(P.mu);
  for (auto& e : P.ents)
    if (e.s && hipStreamQuery(e.s) == hipSuccess) {  // never wait: a gated grid may be parked for good
      hipStreamDestroy(e.s);
      e.s = nullptr;
    }
}
void half_mask(int h, uint32_t m[8]);
hipStream_t masked_acquire_key(const uint32_t m[8], uint32_t key, double load = 0) {
  int dev = 0;
  hipGetDevice(&dev);
  auto create = [](const uint32_t* mm) -> hipStream_t {
    hipStream_t s = nullptr;
    return hipExtStreamCreateWithCUMask(&s, 8, const_cast<uint32_t*>(mm)) == hipSuccess ? s : nullptr;
  };
  uint32_t mc[8], mm[8];
  half_mask(0, mc);
  half_mask(1, mm);
  const uint32_t* masks[2] = {mc, mm};
  masked_pool().prealloc(dev, masks, kPlan, kPlanLen, create);
  return masked_pool().acquire(dev, m, key, create, load);
}
hipStream_t masked_acquire(const uint32_t m[8]) { return masked_acquire_key(m, 0); }
void masked_release(const uint32_t*, hipStream_t s) { masked_pool().release(s); }
void se_cu_mask(const u32 se_bits[kXcds], uint32_t m[8]);

// CU mask of one half of every XCD.  hipExtStreamCreateWithCUMask bit b
// selects logical CU b/8 of XCD b%8 (an XCD left with no bit runs
// unrestricted), and logical CU i sits on shader engine i%4, so half h is the
// bits whose SE is 2h or 2h+1 (measured: scripts/interfere.py census map).
void half_mask(int h, uint32_t m[8]) {
  for (int w = 0; w < 8; ++w) m[w] = 0;
  for (int b = 0; b < 256; ++b)
    if ((((b / 8) % 4) >> 1) == h) m[b / 32] |= 1u << (b % 32);
}
hipStream_t make_half_stream(int h) {
  uint32_t m[8];
  half_mask(h, m);
  return masked_acquire(m);
}

// CU mask of a set of (XCD, SE) partitions: bit b = logical CU b/8 of XCD
// b%8, which sits on SE (b/8)%4.  se_bits[x] = SEs of XCD x in the set.
void se_cu_mask(const u32 se_bits[kXcds], uint32_t m[8]) {
  for (int w = 0; w < 8; ++w) m[w] = 0;
  for (int b = 0; b < 256; ++b)
    if (se_bits[b % 8] & (1u << ((b / 8) % 4))) m[b / 32] |= 1u << (b % 32);
}

struct Runner {
  GpuCtx* ctx;
  gpbs_runner_cfg_t cfg;
  hipStream_t stream = nullptr;
  hipStream_t half_stream[2] = {nullptr, nullptr};  // spatial mode: CU-masked to one half
  // SE-exclusive mode: streams CU-masked to the class half the tenant
  // owns.  A workgroup of a full-GPU grid that lands on a
  // foreign SE cannot just exit: it may have to wait for that SE's owner to
  // free resources before it is even dispatched, and the kernel -- and the
  // next one on the stream -- completes only after it has.  Confining the
  // grid to the owned CUs removes that coupling (GATE_SE still revokes).
  hipStream_t se_stream[2] = {nullptr, nullptr};  // SEs {0,1} / {2,3} of every XCD (latency lane only)
  hipStream_t key_stream = nullptr;  // gated SE mode: the masked queue of the layout it holds (shared by key)
  // Units launched on a queue this runner has since given back (a layout
  // change) may still run: an event recorded on the old queue at the switch,
  // waited for at stop before the hold words and queue memory are released.
  std::vector<hipEvent_t> retired_ev;
  void retire_stream(hipStream_t s) {
    for (size_t i = 0; i < retired_ev.size();)  // drop the ones already passed
      if (hipEventQuery(retired_ev[i]) == hipSuccess) {
        hipEventDestroy(retired_ev[i]);
        retired_ev[i] = retired_ev.back();
        retired_ev.pop_back();
      } else {
        ++i;
      }
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      hipStreamSynchronize(s);
      return;
    }
    hipEventRecord(e, s);
    retired_ev.push_back(e);
  }
  void drain_retired() {
    for (hipEvent_t e : retired_ev) {
      hipEventSynchronize(e);
      hipEventDestroy(e);
    }
    retired_ev.clear();
  }
  uint32_t key_bits = 0;             // ... its key: the owned (XCD, SE) partition set
  int key_half = -1;
  double key_load = 0;               // launches / s it acquired key_stream with
  int64_t rate_t0 = 0;               // dispatch-rate window of the last layout
  uint64_t rate_l0 = 0;
  int cur_grid = 0;  // grid for the stream pick_stream chose (0: kernel default)
  WorkQueue* d_q = nullptr;  // ring of depth+1 queues
  u32* h_status = nullptr;   // pinned status words
  int nq = 0;
  std::thread th;
  std::mutex mu;
  std::condition_variable cv, idle_cv;
  int64_t pending = 0;   // units submitted but not launched
  int64_t inflight = 0;
  bool stop = false;
  std::deque<int64_t> submit_times;
  gpbs_runner_stats_t st{};
  std::vector<int64_t> lats;
  hipEvent_t ev[16];
  int err = 0;
  // latency hold raised by the unit of queue slot qi (generation + 1; 0: none)
  uint64_t q_hold[16] = {};

  void hold_drop(int qi) {
    if (q_hold[qi]) {
      hold_release(ctx, q_hold[qi] - 1);
      q_hold[qi] = 0;
    }
  }

  // phase-changing tenant: fresh units use the alternate workload while
  // `phase` is 1; q_alt[qi] = workload of the unit in queue slot qi
  std::atomic<int> phase{0};
  uint8_t q_alt[16] = {};
  int cur_alt = 0;  // workload of the unit being launched
  // all-reduce tenant: collective sequence number of the unit in each queue
  // slot (fresh units take the next one; a relaunch keeps its own)
  u32 q_seq[16] = {};
  u32 coll_seq = 0;
  int64_t q_t0[16] = {};  // first launch of the unit in each queue slot (all-reduce relaunch bound)

  struct Work {
    int kind, M, N, K, chunk;
    unsigned long long bytes;
    void *a, *b, *c;
  };
  static int coll_timeout_ms(const Work& w) { return w.K > 0 ? w.K : 5000; }
  Work work(int alt) const {
    if (alt && cfg.alt_kind)
      return Work{cfg.alt_kind, cfg.alt_M, cfg.alt_N, cfg.alt_K, cfg.alt_chunk_bytes, cfg.alt_bytes,
                  cfg.alt_a, cfg.alt_b, cfg.alt_c};
    return Work{cfg.kind, cfg.M, cfg.N, cfg.K, cfg.chunk_bytes, cfg.bytes, cfg.a, cfg.b, cfg.c};
  }

  static u32 unit_total(const Work& w) {
    switch (w.kind) {
      case K_ALLREDUCE: {  // chunks of this rank's slice (M = world, N = rank)
        const u64 n8 = w.bytes / 16, chunk8 = (u64)w.chunk / 16, per = (n8 + w.M - 1) / w.M;
        const u64 lo = (u64)w.N * per, hi = std::min(lo + per, n8);
        return hi > lo ? (u32)((hi - lo + chunk8 - 1) / chunk8) : 0u;
      }
      case K_GEMM: return (u32)gpbs_hip_gemm_units(w.M, w.N);
      case K_STREAM:
      case K_REDUCE: return (u32)((w.bytes + w.chunk - 1) / w.chunk);
      case K_GEMV: return (u32)((w.M + 15) / 16);
    }
    return 0;
  }

  // Spatial mode: launch on the stream masked to the CU half the tenant holds
  // (class pinning keeps a classified tenant on one half); a tenant holding
  // both halves or none (yet) launches unmasked and gates per workgroup.
  // The mask is quantised to the two class halves (SEs {0,1} / {2,3} of every
  // XCD), so a runner creates at most two masked streams, once, and keeps
  // them for its lifetime: every CU mask is a hardware queue of its own, and
  // past the hardware's queue slots the scheduler time-multiplexes queues in
  // ~10 ms slices (measured: arbitrary per-(XCD, SE) masks over four runners
  // collapsed even ungated co-runs to 0.42; destroying and re-creating the
  // masked streams at every policy change added ~10 ms stalls that grew run
  // after run).  An owned set that fits neither half (work-conserving steals
  // across classes) launches unmasked and gates per workgroup.
  hipStream_t pick_se_stream() {
    u32 any = 0, bits = 0;
    for (int x = 0; x < kXcds; ++x)
      for (int e = 0; e < kCtx; ++e)
        if ((__atomic_load_n(&ctx->h_table->owner[kCtx * x + e], __ATOMIC_ACQUIRE) & kOwnerMask) == (u32)cfg.tenant) {
          any |= 1u << e;
          bits |= 1u << (kCtx * x + e);
        }
    const int half = (any & ~0x3u) == 0 ? 0 : ((any & ~0xCu) == 0 ? 1 : -1);
    if (!any || half < 0) return stream;
    if (!key_stream || bits != key_bits || half != key_half) {  // a new layout: its queue (shared with co-sharers)
      uint32_t m[8];
      se_half_mask(half, m);
      if (key_stream) {
        retire_stream(key_stream);
        masked_pool().release(key_stream, key_load);
      }
      // this runner's dispatch rate since its last layout change weights the
      // pipe choice (MaskedPoolCore::pipe_cost)
      const int64_t tnow = mono_ns();
      key_load = rate_t0 && tnow > rate_t0 ? (double)(st.launches - rate_l0) * 1e9 / (double)(tnow - rate_t0) : 0.0;
      rate_t0 = tnow;
      rate_l0 = st.launches;
      key_stream = masked_acquire_key(m, bits, key_load);
      key_bits = bits;
      key_half = half;
      if (!key_stream) return stream;
    }
    cur_grid = (work(cur_alt).kind == K_GEMV) ? 0 : 128;  // one persistent WG per CU of the half
    return key_stream;
  }

  bool shared() const { return cfg.gate && ctx->share.load(std::memory_order_acquire); }

  static void se_half_mask(int half, uint32_t m[8]) {
    u32 bits[kXcds];
    for (int x = 0; x < kXcds; ++x) bits[x] = half ? 0xCu : 0x3u;
    se_cu_mask(bits, m);
  }
  hipStream_t half_se_stream(int half) {
    if (!se_stream[half]) {
      uint32_t m[8];
      if (se_stream[half ^ 1]) {  // hold one masked queue per runner at a time
        se_half_mask(half ^ 1, m);
        retire_stream(se_stream[half ^ 1]);
        masked_release(m, se_stream[half ^ 1]);
        se_stream[half ^ 1] = nullptr;
      }
      se_half_mask(half, m);
      se_stream[half] = masked_acquire(m);
      if (!se_stream[half]) return stream;
    }
    return se_stream[half];
  }

  hipStream_t pick_stream() {
    cur_grid = 0;
    const bool se = __atomic_load_n(&ctx->se_mode, __ATOMIC_ACQUIRE);
    const int lh = __atomic_load_n(&ctx->lat_half, __ATOMIC_ACQUIRE);
    if (cfg.priority > 0 && !cfg.gate && lh >= 0) return half_se_stream(lh & 1);  // latency lane
    if (shared()) return stream;  // class-share mode: full-GPU grid, co-resident
    if (cfg.gate && se) return pick_se_stream();
    if (!ctx->spatial || !cfg.gate) return stream;
    // Masked only if every XCD the tenant holds is split and it holds the
    // same half of all of them; otherwise unmasked + per-workgroup gating.
    int half = -1;
    for (int x = 0; x < kXcds; ++x) {
      const u32 w0 = __atomic_load_n(&ctx->h_table->owner[kCtx * x], __ATOMIC_ACQUIRE);
      const u32 w1 = __atomic_load_n(&ctx->h_table->owner[kCtx * x + 1], __ATOMIC_ACQUIRE);
      const bool h0 = (w0 & kOwnerMask) == (u32)cfg.tenant, h1 = (w1 & kOwnerMask) == (u32)cfg.tenant;
      if (!h0 && !h1) continue;
      if ((h0 && h1) || !(w0 & kSplitBit)) return stream;
      const int k = h0 ? 0 : 1;
      if (half >= 0 && half != k) return stream;
      half = k;
    }
    if (half < 0) return stream;
    const int k = half;
    if (!half_stream[k]) half_stream[k] = make_half_stream(k);
    return half_stream[k] ? half_stream[k] : stream;
  }

  int launch(int qi, hipStream_t stream) {
    WorkQueue* q = d_q + qi;
    const Work w = work(q_alt[qi]);
    const int tm = __atomic_load_n(&ctx->table_mode, __ATOMIC_ACQUIRE);
    const bool dev = tm != 0;
    const void* tab = tm == 1 ? (const void*)ctx->d_table : tm == 2 ? (const void*)ctx->b_table : (const void*)ctx->h_table;
    const bool gate = cfg.gate && !ctx->share.load(std::memory_order_acquire);
    // memory-class tenants pause at unit boundaries while a latency request
    // is in flight (only where the host can write the hold word: host / BAR table)
    const bool hold = gate && ctx->hold_enable && tm != 1 && w.kind != K_GEMV && ctx->engine &&
                      ctx->cls_cache[cfg.tenant].load(std::memory_order_relaxed) == 1;
    const unsigned mode = (gate ? (cfg.gate == 2 ? GATE_PARK : GATE_TABLE) : GATE_NONE) | (dev ? GATE_DEVTABLE : 0) |
                          (gate && ctx->spatial ? GATE_SPATIAL : 0) |
                          (gate && __atomic_load_n(&ctx->se_mode, __ATOMIC_ACQUIRE) ? GATE_SE : 0) |
                          (cfg.priority > 0 && ctx->waveprio ? GATE_WAVEPRIO : 0) | (hold ? GATE_HOLD : 0);
    const unsigned me = (unsigned)cfg.tenant;
    __atomic_store_n(&h_status[qi], 0u, __ATOMIC_RELEASE);
    st.launches++;
    const int grid = cfg.grid ? cfg.grid : cur_grid;
    switch (w.kind) {
      case K_GEMM:
        return gpbs_hip_gemm_bf16(w.a, w.b, w.c, w.M, w.N, w.K, q, tab, mode, me, ctx->d_cnt, &h_status[qi], grid,
                                  stream);
      case K_STREAM:
        return gpbs_hip_stream_copy(w.a, w.c, w.bytes, (unsigned)w.chunk, q, tab, mode, me, ctx->d_cnt,
                                    &h_status[qi], grid, stream);
      case K_REDUCE:
        return gpbs_hip_reduce_bf16(w.a, w.b, w.c, w.bytes, (unsigned)w.chunk, q, tab, mode, me, ctx->d_cnt,
                                    &h_status[qi], grid, stream);
      case K_GEMV:
        return gpbs_hip_gemv_bf16(w.a, w.b, w.c, w.M, w.K, q, tab, mode, me, ctx->d_cnt, &h_status[qi], grid,
                                  stream);
      case K_ALLREDUCE:  // K = barrier timeout (ms) -> 100 MHz wall-clock ticks; a 1 ms wait yields the GPU
        return gpbs_hip_allreduce(w.a, q_seq[qi], w.bytes, (unsigned)w.chunk, q, tab, mode, me, ctx->d_cnt,
                                  &h_status[qi], grid, (unsigned long long)coll_timeout_ms(w) * 100000ull,
                                  100000ull, stream);
    }
    return -22;
  }

  bool owns_any() {
    if (!cfg.gate || shared()) return true;
    for (int x = 0; x < kXcds * kCtx; ++x)
      if ((__atomic_load_n(&ctx->h_table->owner[x], __ATOMIC_ACQUIRE) & kOwnerMask) == (u32)cfg.tenant) return true;
    return false;
  }

  // Switch-cost measurement (round 6).  drain: a unit revoked mid-way is
  // watched while the runner waits for ownership, so the moment its grid has
  // left is seen within ~25 us (the runner's own loop only looks at it once
  // it owns a partition again); ramp: the first launch after the wait.
  int wo_qi = -1;               // in-flight unit to watch while waiting (the pipeline's oldest)
  int64_t q_l0[16] = {};        // launch time of the unit in each queue slot (this launch)
  int64_t drain_seen_rv = 0;    // the revocation whose drain was recorded
  int64_t ramp_from = 0;        // wait_owner blocked since here: the next launch closes a ramp
  static void ewma(std::atomic<int64_t>& a, std::atomic<uint64_t>& n, int64_t v) {
    const int64_t o = a.load(std::memory_order_relaxed);
    a.store(n.load(std::memory_order_relaxed) ? o + (v - o) / 8 : v, std::memory_order_relaxed);
    n.fetch_add(1, std::memory_order_relaxed);
  }
  // The unit in queue slot qi has completed its grid at `now`: a revocation
  // drain if it was interrupted (unfinished) by a publish after its launch.
  void note_drain(int qi, int64_t now) {
    if (cfg.tenant < 0 || cfg.tenant >= kMaxTenants) return;
    const int64_t rv = ctx->revoke_ns[cfg.tenant].load(std::memory_order_relaxed);
    if (!rv || rv == drain_seen_rv || rv < q_l0[qi] || now < rv) return;
    const u32 s = __atomic_load_n(&h_status[qi], __ATOMIC_ACQUIRE);
    if ((s & 0x80000000u) && (s & 0x3fffffffu) >= unit_total(work(q_alt[qi]))) return;  // finished, not revoked
    drain_seen_rv = rv;
    const int64_t dr = now - rv;
    if (dr >= 1000000000) return;
    st.drain_sum_ns += dr;
    st.drain_count++;
    if (dr > st.drain_max_ns) st.drain_max_ns = dr;
    ewma(ctx->swc_drain_ns[cfg.tenant], ctx->swc_drain_n[cfg.tenant], dr);
  }
  void note_ramp(int64_t now) {
    if (!ramp_from || cfg.tenant < 0 || cfg.tenant >= kMaxTenants) return;
    const int64_t g = ctx->grant_ns[cfg.tenant].load(std::memory_order_relaxed);
    if (g >= ramp_from && now >= g && now - g < 1000000000)
      ewma(ctx->swc_ramp_ns[cfg.tenant], ctx->swc_ramp_n[cfg.tenant], now - g);
    ramp_from = 0;
  }

  void wait_owner() {
    if (owns_any()) return;
    st.waits_owner++;
    const int64_t t0 = mono_ns();
    ramp_from = t0;
    int watch = wo_qi;
    std::unique_lock<std::mutex> lk(ctx->mu);
    while (!stop && !owns_any()) {
      ctx->cv.wait_for(lk, std::chrono::microseconds(watch >= 0 ? 25 : 200));
      if (watch >= 0) {
        lk.unlock();
        if (hipEventQuery(ev[watch]) != hipErrorNotReady) {
          note_drain(watch, mono_ns());
          watch = -1;
        }
        lk.lock();
      }
    }
    st.wait_owner_ns += mono_ns() - t0;
  }

  void engine_wake(bool on) {
    if (!cfg.engine_wake || !ctx->engine) return;
    if (on)
      gpbs_slot_wake(ctx->engine, cfg.tenant, -1);
    else
      gpbs_slot_block(ctx->engine, cfg.tenant, -1);
  }

  void loop() {
    hipSetDevice(ctx->device);
    struct Fl {
      int qi;
      int ev;
    };
    std::deque<Fl> fl;
    int next_q = 0;
    std::vector<char> q_busy(nq, 0);
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || pending > 0; });
        if (stop) break;
      }
      engine_wake(true);
      const int64_t batch_t0 = mono_ns();
      if (!st.first_start_ns) st.first_start_ns = batch_t0;
      std::deque<int> relaunch;  // queue indices with revoked (unfinished) units
      for (;;) {
        // Fill the pipeline.
        for (;;) {
          if ((int)fl.size() >= cfg.depth) break;
          int qi = -1;
          bool fresh = false;
          if (!relaunch.empty()) {
            qi = relaunch.front();
          } else {
            std::lock_guard<std::mutex> g(mu);
            if (pending <= 0) break;
            for (int k = 0; k < nq; ++k) {
              int cand = (next_q + k) % nq;
              if (!q_busy[cand]) {
                qi = cand;
                break;
              }
            }
            if (qi < 0) break;
            fresh = true;
          }
          wo_qi = fl.empty() ? -1 : fl.front().qi;
          wait_owner();
          if (stop) break;
          if (fresh) {
            q_alt[qi] = (uint8_t)(cfg.alt_kind && phase.load(std::memory_order_acquire));
            q_seq[qi] = coll_seq++;
            q_t0[qi] = mono_ns();
          }
          cur_alt = q_alt[qi];
          hipStream_t stream = pick_stream();
          if (fresh) {
            std::lock_guard<std::mutex> g(mu);
            pending--;
            inflight++;
            next_q = (qi + 1) % nq;
            q_busy[qi] = 1;
          } else {
            relaunch.pop_front();
            st.relaunches++;
            // resume the same queue (its last workgroup out already cleared
            // the exit bookkeeping: no fill kernel here)
          }
          if (cfg.priority > 0 && ctx->hold_enable && fresh && !q_hold[qi]) q_hold[qi] = hold_acquire(ctx) + 1;
          q_l0[qi] = mono_ns();
          note_ramp(q_l0[qi]);
          if (launch(qi, stream) != 0) err = -5;
          const int e = qi;  // one event per queue slot
          hipEventRecord(ev[e], stream);
          fl.push_back({qi, e});
        }
        if (fl.empty()) {
          std::lock_guard<std::mutex> g(mu);
          if (pending <= 0 && relaunch.empty()) break;
          continue;
        }
        Fl f = fl.front();
        fl.pop_front();
        while (hipEventQuery(ev[f.ev]) == hipErrorNotReady) {
          if (stop) break;
          std::this_thread::yield();
        }
        const u32 s = __atomic_load_n(&h_status[f.qi], __ATOMIC_ACQUIRE);
        const u32 done = s & 0x3fffffffu;
        const Work fw = work(q_alt[f.qi]);
        const bool unfinished = !((s & 0x80000000u) && done >= unit_total(fw));
        // all-reduce: a unit still unfinished after the barrier timeout
        // (counted over its relaunches: the kernel yields every 1 ms) fails too
        const bool coll_late = fw.kind == K_ALLREDUCE && unfinished &&
                               mono_ns() - q_t0[f.qi] > (int64_t)coll_timeout_ms(fw) * 1000000;
        if (((s & 0x80000000u) && (s & 0x40000000u)) || coll_late) {
          // all-reduce tenant: a peer barrier timed out (a peer is gone or
          // stalled for seconds) -- fail the runner instead of retrying
          std::fprintf(stderr, "[gpbs-hip] tenant %d: collective unit %u timed out waiting for its peers\n",
                       cfg.tenant, q_seq[f.qi]);
          err = -110;
          hold_drop(f.qi);
          std::lock_guard<std::mutex> g(mu);
          q_busy[f.qi] = 0;
          inflight--;
          pending = 0;
          if (!submit_times.empty()) submit_times.pop_front();
        } else if ((s & 0x80000000u) && done >= unit_total(work(q_alt[f.qi]))) {
          hold_drop(f.qi);
          const int64_t t = mono_ns();
          std::lock_guard<std::mutex> g(mu);
          q_busy[f.qi] = 0;
          inflight--;
          st.units_done++;
          st.units_alt += q_alt[f.qi];
          st.last_done_ns = t;
          if (!submit_times.empty()) {
            const int64_t lat = t - submit_times.front();
            submit_times.pop_front();
            st.lat_sum_ns += lat;
            st.lat_count++;
            if (lat > st.lat_max_ns) st.lat_max_ns = lat;
            if (lats.size() < (1u << 20)) lats.push_back(lat);
          }
        } else {
          relaunch.push_back(f.qi);  // revoked mid-unit: resume when owned
          // seen at once (the runner did not wait for ownership in between;
          // otherwise wait_owner recorded it)
          note_drain(f.qi, mono_ns());
        }
        if (stop) break;
      }
      st.busy_ns += mono_ns() - batch_t0;
      {
        std::lock_guard<std::mutex> g(mu);
        if (pending <= 0 && inflight <= 0) {
          engine_wake(false);
          idle_cv.notify_all();
        }
      }
      if (stop) break;
    }
    hipStreamSynchronize(stream);
    for (hipStream_t h : half_stream)
      if (h) hipStreamSynchronize(h);
    for (hipStream_t h : se_stream)
      if (h) hipStreamSynchronize(h);
    if (key_stream) hipStreamSynchronize(key_stream);
    drain_retired();
    for (int qi = 0; qi < nq; ++qi) hold_drop(qi);  // stopped with latency units in flight
    std::lock_guard<std::mutex> g(mu);
    idle_cv.notify_all();
  }
};

}  // namespace

extern "C" {

void* gpbs_gpu_ctx_create(int device, int part_base, int table_mode, int nctx) {
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  auto* c = new GpuCtx;
  c->device = device;
  c->part_base = part_base;
  c->table_mode = table_mode;
  c->nctx = nctx < 1 ? 1 : (nctx > kCtx ? kCtx : nctx);
  std::memset(c->last_delta, 0, sizeof(c->last_delta));
  std::memset(c->own_ns, 0, sizeof(c->own_ns));
  std::memset(c->own_base, 0, sizeof(c->own_base));
  for (auto& k : c->cls_cache) k.store(-1, std::memory_order_relaxed);
  c->hwc_tokens = c->hwc_bucket;
  bool ok = hipHostMalloc((void**)&c->h_table, sizeof(PartTable), hipHostMallocCoherent | hipHostMallocMapped) ==
            hipSuccess;
  // the modeled counter block: host-readable fine-grained VRAM where the
  // system has it (bar_read, no copy kernel), device memory otherwise
  c->d_cnt = (u64*)finegrained_alloc(device, sizeof(u64) * kMaxTenants * kXcds * kNumPmc);
  c->cnt_bar = c->d_cnt != nullptr;
  if (!c->cnt_bar) ok = ok && hipMalloc((void**)&c->d_cnt, sizeof(u64) * kMaxTenants * kXcds * kNumPmc) == hipSuccess;
  ok = ok && hipMalloc((void**)&c->d_prev, sizeof(u64) * kMaxTenants * kXcds * kNumPmc) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_blk, sizeof(u64) * kMaxTenants * kXcds * kNumPmc, hipHostMallocDefault) ==
                 hipSuccess;
  ok = ok && hipEventCreateWithFlags(&c->blk_ev, hipEventDisableTiming) == hipSuccess;
  c->blk_prev.assign((size_t)kMaxTenants * kXcds * kNumPmc, 0);
  c->red_prev.assign((size_t)kMaxTenants * kXcds * kNumPmc, 0);
  c->snap_blk.assign((size_t)kMaxTenants * kXcds * kNumPmc, 0);
  c->snap_se.assign((size_t)kXcds * kCtx * kNumPmc, 0);
  c->snap_x.assign((size_t)kXcds * kNumPmc, 0);
  c->snap_own.assign((size_t)kMaxTenants * kXcds * kCtx, 0);
  c->snap_chg.assign((size_t)kXcds * kCtx, 0);
  hwc_attr_prev_init(c->hst);
  ok = ok && hipHostMalloc((void**)&c->h_ain, sizeof(HwcAttrIn), hipHostMallocMapped) == hipSuccess;
  ok = ok && hipMalloc((void**)&c->d_ain, sizeof(HwcAttrIn)) == hipSuccess;
  c->f_ain = (HwcAttrIn*)finegrained_alloc(device, sizeof(HwcAttrIn));
  ok = ok && hipHostMalloc((void**)&c->h_aout, sizeof(HwcAttrOut), hipHostMallocMapped) == hipSuccess;
  ok = ok && hipMalloc((void**)&c->d_ast, sizeof(HwcAttrPrev)) == hipSuccess;
  ok = ok && hipMemcpy(c->d_ast, &c->hst, sizeof(HwcAttrPrev), hipMemcpyHostToDevice) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&c->attr_ev, hipEventDisableTiming) == hipSuccess;
  if (!c->cnt_bar) ok = ok && hipMemset(c->d_cnt, 0, sizeof(u64) * kMaxTenants * kXcds * kNumPmc) == hipSuccess;
  ok = ok && hipMemset(c->d_prev, 0, sizeof(u64) * kMaxTenants * kXcds * kNumPmc) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_out, sizeof(u64) * 4 * kMaxTenants, hipHostMallocMapped) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_ids, sizeof(int) * kMaxTenants, hipHostMallocMapped) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_out2, sizeof(u64) * 4 * kMaxTenants, hipHostMallocMapped) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_ids2, sizeof(int) * kMaxTenants, hipHostMallocMapped) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&c->red_ev, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&c->adapt_ev, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_states, sizeof(gpbs_adapt_state_t) * kMaxTenants, hipHostMallocMapped) ==
                 hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_spin, sizeof(u64) * 2 * kMaxTenants, hipHostMallocMapped) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_dirs, sizeof(int) * kMaxTenants, hipHostMallocMapped) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&c->h_adelta, sizeof(u64) * 4 * kMaxTenants, hipHostMallocMapped) == hipSuccess;
  for (auto& B : c->abuf) {
    ok = ok && hipHostMalloc((void**)&B.st, sizeof(gpbs_adapt_state_t) * kMaxTenants, hipHostMallocMapped) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&B.delta, sizeof(u64) * 4 * kMaxTenants, hipHostMallocMapped) == hipSuccess;
    ok = ok && hipHostMalloc((void**)&B.spin, sizeof(u64) * 2 * kMaxTenants, hipHostMallocMapped) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&B.ev, hipEventDisableTiming) == hipSuccess;
  }
  int lo = 0, hi = 0;
  hipDeviceGetStreamPriorityRange(&lo, &hi);
  ok = ok && hipStreamCreateWithPriority(&c->sched_stream, hipStreamNonBlocking, hi) == hipSuccess;
  // the sampler's stream too: a hardware queue created later, between two
  // CU-masked ones, would shift the masked pool's pipe arithmetic (MaskedPoolCore)
  ok = ok && hipStreamCreateWithFlags(&c->hwc_stream, hipStreamNonBlocking) == hipSuccess;
  ok = ok && hipMalloc((void**)&c->d_table, sizeof(PartTable)) == hipSuccess;
  if (!ok) {
    fprintf(stderr, "[gpbs-hip] ctx_create failed on device %d\n", device);
    return nullptr;
  }
  std::memset(c->h_table, 0, sizeof(PartTable));
  for (int x = 0; x < kXcds * kCtx; ++x) {
    c->h_table->owner[x] = kNoOwner;
    c->pending[x] = kNoOwner;
    c->last_real[x] = kNoOwner;
  }
  hipMemcpy(c->d_table, c->h_table, sizeof(PartTable), hipMemcpyHostToDevice);
  // Warm the scheduler kernels once: the first launch of a kernel loads its
  // code object (~3 ms), which must not land inside the first metric tick or
  // table publish under the engine lock (seen as the 3 ms tails of the
  // gpbs:metric_tick / gpbs:publish roctx ranges).
  c->h_ids[0] = -1;
  gpbs_hip_partition_switch(c->d_table, 0, c->pending, c->sched_stream);
  gpbs_hip_counter_reduce(c->d_cnt, c->d_prev, c->h_ids, 1, c->h_out, c->sched_stream);
  hipStreamSynchronize(c->sched_stream);
  return c;
}

void gpbs_gpu_ctx_destroy(void* p) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return;
  hipSetDevice(c->device);
  if (c->hwc_th.joinable()) {  // the sampler reads d_cnt: stop it first
    c->hwc_stop = true;
    c->hwc_th.join();
  }
  hipDeviceSynchronize();
  if (c->engine && !c->muxed) {
    gpbs_set_actuator_ops(c->engine, nullptr);
    gpbs_set_counter_ops(c->engine, nullptr);
  }
  hipStreamDestroy(c->sched_stream);
  hipHostFree(c->h_table);
  if (c->cnt_bar)
    hsa_amd_memory_pool_free(c->d_cnt);
  else
    hipFree(c->d_cnt);
  hipFree(c->d_prev);
  hipHostFree(c->h_out);
  if (c->hwc_stream) hipStreamDestroy(c->hwc_stream);
  if (c->h_blk) hipHostFree(c->h_blk);
  if (c->blk_ev) hipEventDestroy(c->blk_ev);
  hipHostFree(c->h_ids);
  hipHostFree(c->h_out2);
  hipHostFree(c->h_ids2);
  hipEventDestroy(c->red_ev);
  if (c->adapt_ev) {
    hipEventSynchronize(c->adapt_ev);
    hipEventDestroy(c->adapt_ev);
  }
  if (c->attr_ev) {
    hipEventSynchronize(c->attr_ev);
    hipEventDestroy(c->attr_ev);
  }
  if (c->h_ain) hipHostFree(c->h_ain);
  if (c->h_aout) hipHostFree(c->h_aout);
  if (c->d_ast) hipFree(c->d_ast);
  if (c->d_ain) hipFree(c->d_ain);
  if (c->f_ain) hsa_amd_memory_pool_free(c->f_ain);
  for (auto& B : c->abuf) {
    if (B.ev) {
      hipEventSynchronize(B.ev);
      hipEventDestroy(B.ev);
    }
    if (B.st) hipHostFree(B.st);
    if (B.delta) hipHostFree(B.delta);
    if (B.spin) hipHostFree(B.spin);
  }
  hipHostFree(c->h_states);
  hipHostFree(c->h_spin);
  hipHostFree(c->h_dirs);
  hipHostFree(c->h_adelta);
  if (c->d_table) hipFree(c->d_table);
  if (c->b_table) hsa_amd_memory_pool_free(c->b_table);
  delete c;
}

// Install the GPU actuator and counter backend on an engine.
int gpbs_gpu_attach(void* p, gpbs_engine_t* e, int device_counters, int device_adapt) {
  GpuCtx* c = (GpuCtx*)p;
  c->engine = e;
  for (auto& B : c->abuf)  // a new engine harvests nothing an old one launched
    if (B.state == 1) B.state = 2;
  gpbs_actuator_ops_t a{};
  a.user = c;
  a.on_switch = act_on_switch;
  a.on_flush = act_on_flush;
  a.on_park = act_on_park;
  gpbs_set_actuator_ops(e, &a);
  gpbs_counter_ops_t k{};
  k.user = c;
  if (device_counters) k.tenant_deltas = ctr_tenant_deltas;
  if (device_adapt == 1) {  // asynchronous: launched by one metric tick, applied by the next
    k.adapt_launch = ctr_adapt_launch;
    k.adapt_harvest = ctr_adapt_harvest;
  } else if (device_adapt == 2) {  // synchronous, bounded poll under the engine lock (round 2)
    k.adapt_batch = ctr_adapt_batch;
  }
  gpbs_set_counter_ops(e, &k);
  return 0;
}

// Fill (do not install) this context's actuator + counter ops, for the
// engine's per-GPU backend mux (gpbs_backend_mux_add): one engine spanning
// several GPUs, one GpuCtx per GPU.  The caller clears the mux before
// destroying the context.
int gpbs_gpu_backend_ops(void* p, gpbs_engine_t* e, gpbs_actuator_ops_t* a, gpbs_counter_ops_t* k,
                         int device_counters) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c || !a || !k) return -22;
  c->engine = e;
  c->muxed = 1;
  *a = gpbs_actuator_ops_t{};
  a->user = c;
  a->on_switch = act_on_switch;
  a->on_flush = act_on_flush;
  a->on_park = act_on_park;
  *k = gpbs_counter_ops_t{};
  k->user = c;
  if (device_counters) k->tenant_deltas = ctr_tenant_deltas;
  return 0;
}

// Issue contexts per XCD used by the attached engine's partitions (1..kCtx).
int gpbs_gpu_set_nctx(void* p, int nctx) {
  GpuCtx* c = (GpuCtx*)p;
  c->nctx = nctx < 1 ? 1 : (nctx > kCtx ? kCtx : nctx);
  return 0;
}

// Switch between the pinned host table (0) and the device table (1).  The
// device copy is re-synchronised before device mode takes effect.
// Drive the scheduler with live hardware counters (gpbs_hwc_* must be
// initialised and started); 0 falls back to the modeled counters.
int gpbs_gpu_set_hwc(void* p, int on) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  if (on && !gpbs_hwc_active()) return -19;
  if (c->hwc_th.joinable()) {
    c->hwc_stop = true;
    c->hwc_th.join();
  }
  c->share.store(0, std::memory_order_release);  // the sampler decides class sharing: none without it
  std::lock_guard<std::mutex> g(c->mu);
  c->hwc = on ? 1 : 0;
  {
    std::lock_guard<std::mutex> sg(c->snap_mu);
    if (c->attr_pending) {  // an attribution still in flight belongs to the old run
      hipEventSynchronize(c->attr_ev);
      c->attr_pending = false;
    }
    c->hw_primed = false;
    c->used_seq = c->snap_seq;
  }
  for (int k = 0; k < kNumPmc; ++k) c->slot_se[k] = on ? gpbs_hwc_slot_per_se(k) : 0;
  if (on) {
    if (!c->hwc_stream && hipStreamCreateWithFlags(&c->hwc_stream, hipStreamNonBlocking) != hipSuccess) return -5;
    c->hwc_stop = false;
    c->hwc_th = std::thread(hwc_loop, c);
  }
  return 0;
}

// hwc stats: samples, mean sample cost (ns), hardware/modeled ratio per slot.
int gpbs_gpu_hwc_stats(void* p, uint64_t* samples, uint64_t* mean_ns, double* ratio4) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  if (samples) *samples = c->hwc_samples;
  if (mean_ns) *mean_ns = c->hwc_samples ? (uint64_t)(c->hwc_ns / (int64_t)c->hwc_samples) : 0;
  if (ratio4)
    for (int k = 0; k < kNumPmc; ++k) ratio4[k] = c->model_sum[k] > 0 ? c->hw_sum[k] / c->model_sum[k] : 0.0;
  return 0;
}

// Attribution quality: max sample cost (ns), and per slot the fraction of
// hardware counts no owner explains.  Slot mask of the SE-resolved slots.
int gpbs_gpu_hwc_quality(void* p, uint64_t* max_ns, double* unatt_frac4, int* se_slots) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  if (max_ns) *max_ns = (uint64_t)c->hwc_ns_max;
  if (unatt_frac4)
    for (int k = 0; k < kNumPmc; ++k) unatt_frac4[k] = c->hw_sum[k] > 0 ? c->unatt[k] / c->hw_sum[k] : 0.0;
  if (se_slots) {
    *se_slots = 0;
    for (int k = 0; k < kNumPmc; ++k) *se_slots |= (c->slot_se[k] && c->se_mode) << k;
  }
  return 0;
}

// Exclusive-ownership windows: set the minimum share (percent) of a sample
// interval one tenant must own a partition for its delta to reach the PBS
// metric (0: every interval, split pro rata).  Returns the previous value;
// frac4 (optional) receives, per slot, the fraction of all hardware counts
// since the last reset that reached the metric.
int gpbs_gpu_hwc_clean(void* p, int pct, double* frac4) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  const int old = c->clean_pct;
  if (pct >= 0) c->clean_pct = std::min(pct, 100);
  if (frac4)
    for (int k = 0; k < kNumPmc; ++k) frac4[k] = c->hw_sum[k] > 0 ? c->metric_sum[k] / c->hw_sum[k] : 0.0;
  return old;
}

// Per-tenant cumulative attributed hardware counts and modeled counts since
// the last reset (PBS slots INST, CYCLES, LLC_REFS, LLC_MISSES).
int gpbs_gpu_hwc_tenant(void* p, int t, double* att4, double* model4) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c || t < 0 || t >= kMaxTenants) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  for (int k = 0; k < kNumPmc; ++k) {
    if (att4) att4[k] = c->att_total[t][k];
    if (model4) model4[k] = c->mod_total[t][k];
  }
  return 0;
}

// Per-tenant cumulative counts that reached the PBS metric (exclusive-
// ownership windows) since the last reset.
int gpbs_gpu_hwc_tenant_metric(void* p, int t, double* m4) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c || t < 0 || t >= kMaxTenants || !m4) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  for (int k = 0; k < kNumPmc; ++k) m4[k] = c->met_total[t][k];
  return 0;
}

// Consume the newest sampler snapshot now (attribution into the per-tenant
// totals and pending deltas) -- what the engine's metric tick does; for
// tools and tests that run without an engine.
int gpbs_gpu_hwc_poll(void* p) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c || !c->hwc) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  return hwc_consume(c, true);
}

// Attribution path counters: kernel launches, ticks that found the previous
// launch still running, host-path attributions.  Returns dev_attr.
int gpbs_gpu_hwc_attr_stats(void* p, uint64_t* launches, uint64_t* busy_skips, uint64_t* host) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  if (launches) *launches = c->attr_launches;
  if (busy_skips) *busy_skips = c->attr_busy_skips;
  if (host) *host = c->attr_host;
  return c->dev_attr;
}

// In-run timing of the device attribution since the last hwc reset: out4 =
// attributions harvested, mean and max k_hwc_attribute duration (ns, the
// kernel's own wall-clock stamps), mean launch -> harvest latency (ns).
int gpbs_gpu_hwc_attr_timing(void* p, uint64_t* out4) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c || !out4) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  const uint64_t n = c->attr_harvested;
  out4[0] = n;
  out4[1] = n ? c->attr_ticks_sum * 10 / n : 0;  // 100 MHz ticks -> ns
  out4[2] = c->attr_ticks_max * 10;
  out4[3] = n ? (uint64_t)(c->attr_lag_sum_ns / (int64_t)n) : 0;
  return 0;
}

// Device attribution on (1) / off (0, host reference); returns the old value.
int gpbs_gpu_set_hwc_device(void* p, int on) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  const int old = c->dev_attr;
  if (on >= 0 && on != old) {
    if (c->attr_pending) {
      hipEventSynchronize(c->attr_ev);
      hwc_fold(c, *c->h_aout, c->mod_inflight, c->pres_inflight, c->t_inflight);
      c->attr_pending = false;
    }
    c->dev_attr = on ? 1 : 0;
    c->hw_primed = false;  // the other path's previous snapshot is stale: re-prime
  }
  return old;
}

// Numerics check of k_hwc_attribute against hwc_attr_host on `iters` random
// snapshot pairs (seeded): max relative difference of the attributed and
// clean deltas and the interval totals.  Stand-alone (no context needed).
// Cost of one attribution (a live-layout snapshot in pinned host memory, as
// on the headline path): out[0] = mean interval per launch over `iters`
// back-to-back launches (hipEvent: kernel + dispatch gap), out[1] = mean host
// round trip of one launch + event wait, out[2] = mean kernel duration from
// the kernel's own entry / exit wall-clock stamps.  0 on success.
// Two pools on one GpuContext, device adapt: pool A launches
// for tenants {1,2}, pool B for {3,4}, interleaved and harvested in both
// orders; every harvest must return the caller's own tenants with the host
// adapt_update's states.  Returns 0, or the first failing step (< 0).
int gpbs_hip_adapt_pools_selftest(int rounds) {
  void* h = gpbs_gpu_ctx_create(0, 0, 0, 4);
  if (!h) return -12;
  GpuCtx* c = (GpuCtx*)h;
  gpbs_adapt_params_t p{};
  p.threshold = 2000;
  p.band_lo = 70;
  p.band_hi = 130;
  p.min_us = 1000;
  p.max_us = 11000;
  p.inc_us = 1000;
  p.dec_us = 2000;
  p.switch_boundary = 9000;
  p.ticks_per_tslice = 3;
  gpbs_adapt_state_t sa[2] = {}, sb[2] = {};
  for (auto* s : {&sa[0], &sa[1], &sb[0], &sb[1]}) {
    s->tslice_us = 1000;
    s->tick_period_us = 333;
    s->window_left = 5;
  }
  const int ia[2] = {1, 2}, ib[2] = {3, 4};
  int rc = 0;
  for (int r = 0; r < rounds && !rc; ++r) {
    uint64_t da[8], db[8], z[2] = {0, 0};
    for (int k = 0; k < 2; ++k) {  // phases that move the quanta: A high-miss, B low-miss, alternating
      const uint64_t inst = 1000000 + 1000 * r + k;
      da[4 * k] = db[4 * k] = inst;
      da[4 * k + 1] = db[4 * k + 1] = 2 * inst;
      da[4 * k + 2] = db[4 * k + 2] = inst / 10;
      da[4 * k + 3] = ((r / 7) & 1) ? inst / 1000 : inst / 20;
      db[4 * k + 3] = ((r / 5) & 1) ? inst / 20 : inst / 1000;
    }
    if (ctr_adapt_launch(c, 2, ia, da, z, z, sa, &p) || ctr_adapt_launch(c, 2, ib, db, z, z, sb, &p)) {
      rc = -1;
      break;
    }
    hipDeviceSynchronize();
    int ta[2] = {ia[0], ia[1]}, tb[2] = {ib[0], ib[1]};
    gpbs_adapt_state_t oa[2], ob[2];
    const bool a_first = r & 1;
    const int na = a_first ? ctr_adapt_harvest(c, 2, ta, oa) : 0;
    const int nb = ctr_adapt_harvest(c, 2, tb, ob);
    const int na2 = a_first ? na : ctr_adapt_harvest(c, 2, ta, oa);
    if (na2 != 2 || nb != 2 || ta[0] != 1 || ta[1] != 2 || tb[0] != 3 || tb[1] != 4) {
      rc = -2;
      break;
    }
    for (int k = 0; k < 2 && !rc; ++k) {
      gpbs_adapt_update(&sa[k], &p, da[4 * k], da[4 * k + 3], 0, 0);
      gpbs_adapt_update(&sb[k], &p, db[4 * k], db[4 * k + 3], 0, 0);
      if (std::memcmp(&sa[k], &oa[k], sizeof(sa[k])) || std::memcmp(&sb[k], &ob[k], sizeof(sb[k]))) rc = -3;
    }
  }
  // a harvest for tenants nobody launched finds nothing
  int tx[2] = {5, 6};
  gpbs_adapt_state_t ox[2];
  if (!rc && ctr_adapt_harvest(c, 2, tx, ox) != -22) rc = -4;
  gpbs_gpu_ctx_destroy(h);
  return rc;
}

int gpbs_hip_hwc_attr_bench(int iters, double* out2) {
  if (iters <= 0 || !out2) return -22;
  HwcAttrIn* in = nullptr;
  HwcAttrIn* d_in = nullptr;
  HwcAttrOut* out = nullptr;
  HwcAttrPrev* d_st = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = 0;
  if (hipHostMalloc((void**)&in, sizeof(HwcAttrIn), hipHostMallocMapped) != hipSuccess ||
      hipMalloc((void**)&d_in, sizeof(HwcAttrIn)) != hipSuccess ||
      hipHostMalloc((void**)&out, sizeof(HwcAttrOut), hipHostMallocMapped) != hipSuccess ||
      hipMalloc((void**)&d_st, sizeof(HwcAttrPrev)) != hipSuccess || hipStreamCreate(&s) != hipSuccess ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
    rc = -12;
  if (rc == 0) {
    static HwcAttrPrev hst;
    hwc_attr_prev_init(hst);
    hipMemcpy(d_st, &hst, sizeof(hst), hipMemcpyHostToDevice);
    std::memset(in, 0, sizeof(HwcAttrIn));
    for (int p = 0; p < kAttrP; ++p) {  // SE-exclusive layout: one owner per partition, 4 tenants
      in->own_cur[(1 + p % 4) * kAttrP + p] = 1000000;
      for (int k = 0; k < kNumPmc; ++k) in->se_cur[p * kNumPmc + k] = 1000 + p * 7 + k;
    }
    for (int k = 0; k < kNumPmc; ++k) in->slot_se[k] = k < 3;
    in->se_mode = 1;
    in->clean_pct = 90;
    in->prime = 0;
    in->nt_hi = 5;  // tenants 1..4 own partitions
    gpbs_hip_hwc_attribute(in, d_in, d_st, out, s);  // warm
    hipStreamSynchronize(s);
    hipEventRecord(e0, s);
    for (int i = 0; i < iters; ++i) gpbs_hip_hwc_attribute(in, d_in, d_st, out, s);
    hipEventRecord(e1, s);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    out2[0] = 1e3 * ms / iters;
    const int64_t t0 = mono_ns();
    double ticks = 0;
    for (int i = 0; i < iters; ++i) {
      gpbs_hip_hwc_attribute(in, d_in, d_st, out, s);
      hipEventRecord(e1, s);
      hipEventSynchronize(e1);
      ticks += (double)(uint32_t)(out->pad[1] - out->pad[0]);
    }
    out2[1] = (double)(mono_ns() - t0) / 1e3 / iters;
    out2[2] = ticks * 0.01 / iters;  // 100 MHz ticks -> us
    if (hipGetLastError() != hipSuccess) rc = -5;
  }
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  if (s) hipStreamDestroy(s);
  if (d_in) hipFree(d_in);
  if (in) hipHostFree(in);
  if (out) hipHostFree(out);
  if (d_st) hipFree(d_st);
  return rc;
}

// One random attribution input (the previous one advanced): most partitions
// with one dominant owner, some time-shared, some idle; every few steps a
// whole idle XCD, another slot layout, co-resident mode, no clean windows, a
// class-share interval; step 0 primes.
}  // extern "C" (a template needs C++ linkage)
template <class Rnd>
static void attr_random_step(HwcAttrIn& in, int it, Rnd& rnd) {
  for (int p = 0; p < kAttrP; ++p) {
    int kind = (int)(rnd() % 8);
    if (it % 4 == 2 && p / kCtx == 5) kind = 7;  // a whole idle XCD (no owner: unexplained counts)
    const int a = 1 + (int)(rnd() % 6), b = 1 + (int)(rnd() % 6);
    const long long span = 1000000;
    for (int t = 0; t < kMaxTenants; ++t) {
      long long add = 0;
      if (kind < 5 && t == a) add = span;
      else if (kind == 5 && t == a) add = span / 2 + (long long)(rnd() % 1000);
      else if (kind == 5 && t == b) add = span / 2;
      else if (kind == 6 && t == a) add = span * 95 / 100;
      in.own_cur[t * kAttrP + p] += add;
    }
    for (int k = 0; k < kNumPmc; ++k) in.se_cur[p * kNumPmc + k] += rnd() % 100000000ull;
  }
  for (int i = 0; i < kXcds * kNumPmc; ++i) in.x_cur[i] += rnd() % 1000000000ull;
  // slot layouts: the default (0-2 per SE, 3 per XCD), slot 2 per XCD (the
  // L2-miss split by XCD-level requests), every slot per SE
  for (int k = 0; k < kNumPmc; ++k) in.slot_se[k] = it % 6 == 1 ? (k < 2) : it % 6 == 5 ? 1u : (k < 3);
  in.se_mode = (it % 5) != 4;
  in.clean_pct = it % 7 == 3 ? 0 : 90;
  in.shared = it % 11 == 10;
  in.prime = it == 0;
  in.nt_hi = it % 3 == 2 ? 0 : 7;  // tenants 1..6 own partitions (0: read every row)
  in.drained = it % 3 == 1 ? (u32)rnd() : (it % 3 == 2 ? 0xFFFFFFFFu : 0u);  // switch-aligned windows
}

extern "C" {

// Host-only properties of hwc_attr_host (no GPU): per counter slot the
// attributed counts plus the unexplained ones add up to the hardware sum
// (out2[0]: worst relative error), and no tenant's clean part exceeds its
// attributed part (out2[1]: worst relative excess).  Returns 0.
int gpbs_hip_hwc_attr_host_check(int seed, int iters, double* out2) {
  static HwcAttrIn in;
  static HwcAttrPrev st;
  static HwcAttrOut o;
  std::memset(&in, 0, sizeof(in));
  hwc_attr_prev_init(st);
  uint64_t r = 0x9E3779B97F4A7C15ull ^ (uint64_t)seed;
  auto rnd = [&]() {
    r ^= r << 13;
    r ^= r >> 7;
    r ^= r << 17;
    return r;
  };
  double cons = 0, excess = 0;
  for (int it = 0; it <= iters; ++it) {
    attr_random_step(in, it, rnd);
    hwc_attr_host(in, st, o);
    if (!o.valid) continue;
    for (int k = 0; k < kNumPmc; ++k) {
      double sum = o.unatt[k];
      for (int t = 0; t < kMaxTenants; ++t) {
        sum += o.add[t][k];
        if (o.add[t][k] > 0) excess = std::max(excess, (o.addc[t][k] - o.add[t][k]) / o.add[t][k]);
      }
      if (o.hw_sum[k] > 0) cons = std::max(cons, std::fabs(sum - o.hw_sum[k]) / o.hw_sum[k]);
    }
  }
  out2[0] = cons;
  out2[1] = excess;
  return 0;
}

// Host check of the metric fold: a tenant whose hardware rates
// differ from its modeled ones by large factors (the measured 24x on
// instructions, 0.13x on L2 traffic) alternates between clean windows and
// stale unclean periods; the calibrated fallback must deliver the hardware
// miss rate (within 10 %), so the tenant keeps its class.  An uncalibrated
// or fresh unclean period is skipped, a sliver never counts.  No HIP call.
// Returns 0 or the number of the first failed check.
int gpbs_hip_hwc_fold_selftest(void) {
  // a fresh context per call (host fields only; nothing here touches the
  // device): the per-tenant period counts, calibration and last clean window
  // start from zero however often the check runs in one process
  std::unique_ptr<GpuCtx> cp(new GpuCtx());
  GpuCtx& c = *cp;
  std::memset(c.last_delta, 0, sizeof(c.last_delta));
  c.clean_pct = 80;
  const int t = 3;
  const double hw_inst = 2.0e6, hw_miss = 6.0e5;                    // 3e4 misses per 1e5: memory class
  const double md_inst = hw_inst / 24.0, md_miss = hw_miss / 0.13;  // what the kernels model
  static HwcAttrOut o;
  static double mod[kMaxTenants][kNumPmc], pres[kMaxTenants];
  auto period = [&](bool clean, double share) {
    std::memset(&o, 0, sizeof(o));
    std::memset(mod, 0, sizeof(mod));
    std::memset(pres, 0, sizeof(pres));
    o.valid = 1;
    const double f = share;
    o.add[t][0] = hw_inst * f;
    o.add[t][1] = hw_inst * f;
    o.add[t][2] = hw_miss * 2 * f;
    o.add[t][3] = hw_miss * f;
    if (clean)
      for (int k = 0; k < kNumPmc; ++k) o.addc[t][k] = o.add[t][k];
    mod[t][0] = md_inst * f;
    mod[t][1] = md_inst * f;
    mod[t][2] = md_miss * 2 * f;
    mod[t][3] = md_miss * f;
    pres[t] = share;
  };
  auto take = [&](double* inst, double* miss) {
    *inst = (double)c.last_delta[t][0];
    *miss = (double)c.last_delta[t][3];
    for (int k = 0; k < kNumPmc; ++k) c.last_delta[t][k] = 0;
  };
  double in = 0, mi = 0;
  int64_t now = 1000000000;
  // 1. unclean before any calibration: skipped, nothing delivered
  period(false, 1.0);
  hwc_fold(&c, o, mod, pres, now);
  take(&in, &mi);
  if (in != 0 || c.t_skipped[t] != 1) return 1;
  const double thr = 20000;
  for (int round = 0; round < 20; ++round) {
    // a clean window (calibrates), then unclean periods: fresh (skipped), stale (fallback), sliver
    now += 11000000;
    period(true, 1.0);
    hwc_fold(&c, o, mod, pres, now);
    take(&in, &mi);
    if (in <= 0 || std::fabs(mi * 1e5 / in - hw_miss * 1e5 / hw_inst) > 1.0) return 2;
    const int64_t stale = (int64_t)c.hwc_stale_us * 1000;
    now += stale / 5;
    period(false, 0.9);
    hwc_fold(&c, o, mod, pres, now);  // a fifth of the staleness after a clean window: skipped
    take(&in, &mi);
    if (in != 0) return 3;
    now += stale;
    period(false, 0.9);
    hwc_fold(&c, o, mod, pres, now);  // past it: stale -> calibrated fallback
    take(&in, &mi);
    if (in <= 0) return 4;
    const double rate = mi * 1e5 / in, want = hw_miss * 1e5 / hw_inst;
    if (std::fabs(rate - want) > 0.1 * want || rate < thr) return 5;  // same class as the clean windows
    period(false, 0.05);
    hwc_fold(&c, o, mod, pres, now + 1000000);  // the edge of another tenure
    take(&in, &mi);
    if (in != 0) return 6;
  }
  if (c.t_clean[t] != 20 || c.t_fallback[t] != 20 || c.t_sliver[t] != 20 || c.t_skipped[t] != 21) return 7;
  return 0;
}

// Host check of hwc_drained_bits: random owner-change times per
// partition around an interval; a bit may be set only when the opening owner
// had held the partition a guard and no change landed in the interval's head,
// and must be set when both hold.  Also the two cases named in the advice:
// a takeover at the head (no bit) and a switch-aligned close at the tail (bit).
// Returns 0 or the number of the first failed check.  No HIP call.
int gpbs_hip_hwc_drained_selftest(int seed, int iters) {
  uint64_t r = 0x2545F4914F6CDD1Dull ^ (uint64_t)seed;
  auto rnd = [&]() {
    r ^= r << 13;
    r ^= r >> 7;
    r ^= r << 17;
    return r;
  };
  int64_t used_chg[kAttrP], snap_chg[kAttrP];
  const int64_t guard = 150000;
  for (int it = 0; it < iters; ++it) {
    const int64_t used_t = 1000000000 + (int64_t)(rnd() % 1000000);
    const int64_t span = (int64_t)(rnd() % 8000000);
    const int64_t snap_t = used_t + span;
    const u32 cp = it % 5 == 4 ? 0u : (it % 2 ? 80u : 90u);
    for (int p = 0; p < kAttrP; ++p) {
      used_chg[p] = used_t - (int64_t)(rnd() % (4 * guard));
      const int kind = (int)(rnd() % 3);  // no change / change in the interval
      snap_chg[p] = kind == 0 ? used_chg[p] : used_t + 1 + (int64_t)(rnd() % (uint64_t)(span + 1));
    }
    const u32 dr = hwc_drained_bits(used_t, snap_t, used_chg, snap_chg, guard, cp);
    for (int p = 0; p < kAttrP; ++p) {
      const bool settled = used_t - used_chg[p] >= guard;
      const bool head = snap_chg[p] > used_t && (snap_chg[p] - used_t) * 100 <= (int64_t)(100 - cp) * span;
      const bool want = span >= 3 * guard && settled && !head;
      if ((((dr >> p) & 1u) != 0) != want) return 1;
    }
  }
  // the advice's two cases, 4 ms interval, clean_pct 80
  for (int p = 0; p < kAttrP; ++p) used_chg[p] = 1000000000 - 2 * guard;
  const int64_t t0 = 1000000000, t1 = t0 + 4000000;
  for (int p = 0; p < kAttrP; ++p) snap_chg[p] = t0 + 300000;  // B takes over 0.3 ms in: B holds 92 %
  if (hwc_drained_bits(t0, t1, used_chg, snap_chg, guard, 80) != 0) return 2;
  for (int p = 0; p < kAttrP; ++p) snap_chg[p] = t1 - guard;  // A's tenure ends one guard before the close
  if (hwc_drained_bits(t0, t1, used_chg, snap_chg, guard, 80) != 0xFFFFFFFFu) return 3;
  return 0;
}

// Measured switch cost of a tenant (round 6): out4 = drain EWMA ns, ramp
// EWMA ns, drains measured, ramps measured.
int gpbs_gpu_switch_cost(void* ctx, int tenant, int64_t* out4) {
  GpuCtx* c = (GpuCtx*)ctx;
  if (!c || tenant < 0 || tenant >= kMaxTenants || !out4) return -22;
  out4[0] = c->swc_drain_ns[tenant].load(std::memory_order_relaxed);
  out4[1] = c->swc_ramp_ns[tenant].load(std::memory_order_relaxed);
  out4[2] = (int64_t)c->swc_drain_n[tenant].load(std::memory_order_relaxed);
  out4[3] = (int64_t)c->swc_ramp_n[tenant].load(std::memory_order_relaxed);
  return 0;
}

// Host check of the 1 ms cadence: a tenant whose clean
// hardware windows come every 10 ms reports every tick in between from its
// modeled counters x its hardware/model ratio -- the delivered miss rate is
// the hardware one (within 10 %), so it keeps its class with ten times the
// metric periods; a clean window of a calibrated tenant only re-anchors the
// ratio (no double report); and a phase change in the model (the tenant
// turns compute-bound) moves the delivered rate below the class threshold
// at the next tick.  The block is a host buffer standing in for the BAR
// mapping.  No HIP call.  Returns 0 or the number of the first failed check.
int gpbs_hip_hwc_cadence_selftest(void) {
  std::unique_ptr<GpuCtx> cp(new GpuCtx());
  GpuCtx& c = *cp;
  std::vector<u64> blk((size_t)kMaxTenants * kXcds * kNumPmc, 0);
  c.d_cnt = blk.data();
  c.cnt_bar = true;
  c.model_cadence = 1;
  c.clean_pct = 80;
  const int t = 3;
  c.cnt_rows = t + 1;
  const double hw_inst = 2.0e6, hw_miss = 6.0e5;  // per ms: 3e4 misses per 1e5 inst (memory class)
  double md_inst = hw_inst / 24.0, md_miss = hw_miss / 0.13;
  auto advance = [&](double ms) {  // the kernels' modeled counts, spread over the 8 XCDs
    for (int x = 0; x < kXcds; ++x) {
      u64* r = &blk[((size_t)t * kXcds + x) * kNumPmc];
      r[0] += (u64)(md_inst * ms / kXcds);
      r[1] += (u64)(md_inst * ms / kXcds);
      r[2] += (u64)(2 * md_miss * ms / kXcds);
      r[3] += (u64)(md_miss * ms / kXcds);
    }
  };
  static HwcAttrOut o;
  static double mod[kMaxTenants][kNumPmc], pres[kMaxTenants];
  auto window = [&](double ms) {  // a clean hardware window over the last `ms`
    std::memset(&o, 0, sizeof(o));
    std::memset(mod, 0, sizeof(mod));
    std::memset(pres, 0, sizeof(pres));
    o.valid = 1;
    o.add[t][0] = o.addc[t][0] = hw_inst * ms;
    o.add[t][1] = o.addc[t][1] = hw_inst * ms;
    o.add[t][2] = o.addc[t][2] = 2 * hw_miss * ms;
    o.add[t][3] = o.addc[t][3] = hw_miss * ms;
    mod[t][0] = mod[t][1] = md_inst * ms;
    mod[t][2] = 2 * md_miss * ms;
    mod[t][3] = md_miss * ms;
    pres[t] = 1.0;
  };
  auto take = [&](double* inst, double* miss) {
    *inst = (double)c.last_delta[t][0];
    *miss = (double)c.last_delta[t][3];
    for (int k = 0; k < kNumPmc; ++k) c.last_delta[t][k] = 0;
  };
  const double want = hw_miss * 1e5 / hw_inst, thr = 20000;
  double in = 0, mi = 0;
  int64_t now = 1000000000;
  cadence_tick(&c);  // primes
  advance(1);
  cadence_tick(&c);  // not calibrated yet: nothing
  take(&in, &mi);
  if (in != 0) return 1;
  window(10);  // the first clean window calibrates and reports (uncalibrated before it)
  hwc_fold(&c, o, mod, pres, now);
  take(&in, &mi);
  if (in <= 0 || std::fabs(mi * 1e5 / in - want) > 1.0) return 2;
  for (int round = 0; round < 10; ++round) {
    for (int k = 0; k < 9; ++k) {  // nine 1 ms ticks between hardware windows: each reports
      advance(1);
      cadence_tick(&c);
      take(&in, &mi);
      if (in <= 0) return 3;
      const double r = mi * 1e5 / in;
      if (std::fabs(r - want) > 0.1 * want || r < thr) return 4;
    }
    advance(1);
    now += 10000000;
    window(10);
    hwc_fold(&c, o, mod, pres, now);  // calibrated: re-anchors only
    take(&in, &mi);
    if (in != 0) return 5;
  }
  if (c.t_model[t] != 90 || c.t_clean[t] != 11) return 6;
  md_miss = md_miss / 100.0;  // the tenant turns compute-bound: the model sees it at once
  advance(1);
  cadence_tick(&c);
  take(&in, &mi);
  if (in <= 0 || mi * 1e5 / in >= thr) return 7;
  c.d_cnt = nullptr;
  return 0;
}

int gpbs_hip_hwc_attr_selftest(int seed, int iters, double* max_rel) {
  HwcAttrIn* in = nullptr;
  HwcAttrIn* d_in = nullptr;
  HwcAttrOut* out = nullptr;
  HwcAttrPrev* d_st = nullptr;
  if (hipHostMalloc((void**)&in, sizeof(HwcAttrIn), hipHostMallocMapped) != hipSuccess ||
      hipMalloc((void**)&d_in, sizeof(HwcAttrIn)) != hipSuccess ||
      hipHostMalloc((void**)&out, sizeof(HwcAttrOut), hipHostMallocMapped) != hipSuccess ||
      hipMalloc((void**)&d_st, sizeof(HwcAttrPrev)) != hipSuccess)
    return -12;
  static HwcAttrPrev hst;
  static HwcAttrOut ref;
  hwc_attr_prev_init(hst);
  hipMemcpy(d_st, &hst, sizeof(hst), hipMemcpyHostToDevice);
  uint64_t r = 0x9E3779B97F4A7C15ull ^ (uint64_t)seed;
  auto rnd = [&]() {
    r ^= r << 13;
    r ^= r >> 7;
    r ^= r << 17;
    return r;
  };
  std::memset(in, 0, sizeof(HwcAttrIn));
  double worst = 0;
  int rc = 0;
  for (int it = 0; it <= iters && rc == 0; ++it) {
    attr_random_step(*in, it, rnd);
    hwc_attr_host(*in, hst, ref);
    if (gpbs_hip_hwc_attribute(in, d_in, d_st, out, nullptr) || hipDeviceSynchronize() != hipSuccess) {
      rc = -5;
      break;
    }
    if (out->valid != ref.valid) rc = -33;
    auto rel = [](double x, double y) {
      const double m = std::max(std::fabs(x), std::fabs(y));
      return m > 0 ? std::fabs(x - y) / m : 0.0;
    };
    for (int t = 0; t < kMaxTenants; ++t)
      for (int k = 0; k < kNumPmc; ++k) {
        worst = std::max(worst, rel(out->add[t][k], ref.add[t][k]));
        worst = std::max(worst, rel(out->addc[t][k], ref.addc[t][k]));
      }
    for (int k = 0; k < kNumPmc; ++k) {
      worst = std::max(worst, rel(out->hw_sum[k], ref.hw_sum[k]));
      worst = std::max(worst, rel(out->unatt[k], ref.unatt[k]));
    }
  }
  if (max_rel) *max_rel = worst;
  hipFree(d_in);
  hipHostFree(in);
  hipHostFree(out);
  hipFree(d_st);
  return rc;
}

// Runtime parameters by name (gpbs.toml [runtime], pbs_amd/core/config.py):
// sets `name` to `value` (value < 0 reads only) and returns the value before,
// or -22 for an unknown name.  Sampler parameters: period_us (tick),
// slow_us (steady-state back-off), duty_pct (background duty cap), burst_ms
// (phase-trigger burst), budget_pct / bucket (token bucket over every
// sample), clean_pct (exclusive-window share), device_attr (attribution on
// the GPU), fallback (calibrated model fallback), stale_us, watch (modeled
// block every tick), align / guard_us / long_us (switch-aligned samples);
// class-share mode: share, probe_every, probe_len.
int gpbs_gpu_param(void* p, const char* name, int value) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c || !name) return -22;
  struct Ent {
    const char* n;
    int* f;
    int lo, hi;
  };
  const Ent tab[] = {
      {"period_us", &c->hwc_period_us, 100, 1000000},   {"slow_us", &c->hwc_slow_us, 0, 10000000},
      {"duty_pct", &c->hwc_duty_pct, 0, 100},           {"burst_ms", &c->hwc_burst_ms, 0, 10000},
      {"budget_pct", &c->hwc_budget_pct, 0, 100},       {"bucket", &c->hwc_bucket, 1, 100000},
      {"clean_pct", &c->clean_pct, 0, 100},             {"device_attr", &c->dev_attr, 0, 1},
      {"fallback", &c->model_fallback, 0, 1},           {"stale_us", &c->hwc_stale_us, 0, 100000000},
      {"watch", &c->hwc_watch, 0, 1},                   {"align", &c->hwc_align, 0, 1},
      {"guard_us", &c->hwc_guard_us, 0, 100000},        {"long_us", &c->hwc_long_us, 0, 100000000},
      {"pair_gap_us", &c->hwc_pair_gap_us, 0, 10000000}, {"measure_ms", &c->hwc_measure_ms, 0, 100000},
      {"share", &c->share_enable, 0, 1},                {"probe_every", &c->probe_every, 0, 1000000},
      {"probe_len", &c->probe_len, 0, 1000000},         {"cadence", &c->model_cadence, 0, 1},
  };
  for (const Ent& e : tab)
    if (std::strcmp(e.n, name) == 0) {
      std::lock_guard<std::mutex> g(c->snap_mu);
      const int old = *e.f;
      if (value >= 0) {
        if (e.f == &c->dev_attr && (value != 0) != (old != 0)) {  // the other path's state is stale: re-prime
          if (c->attr_pending) {
            hipEventSynchronize(c->attr_ev);
            hwc_fold(c, *c->h_aout, c->mod_inflight, c->pres_inflight, c->t_inflight);
            c->attr_pending = false;
          }
          c->hw_primed = false;
        }
        *e.f = std::max(e.lo, std::min(e.hi, value));
        if (e.f == &c->hwc_bucket || e.f == &c->hwc_budget_pct) c->hwc_tokens = c->hwc_bucket;
      }
      return old;
    }
  return -22;
}

int gpbs_gpu_hwc_reset(void* p) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  std::memset(c->att_total, 0, sizeof(c->att_total));
  std::memset(c->mod_total, 0, sizeof(c->mod_total));
  std::memset(c->hw_sum, 0, sizeof(c->hw_sum));
  std::memset(c->model_sum, 0, sizeof(c->model_sum));
  std::memset(c->unatt, 0, sizeof(c->unatt));
  std::memset(c->metric_sum, 0, sizeof(c->metric_sum));
  std::memset(c->met_total, 0, sizeof(c->met_total));
  c->share_base = c->snap_share;
  c->hwc_ns = c->hwc_ns_max = 0;
  c->measure_reqs = 0;
  c->hwc_samples = 0;
  c->hwc_slow_samples = 0;
  c->hwc_period_sum_ns = 0;
  c->hwc_burst_samples = 0;
  c->hwc_triggers = 0;
  c->hwc_denied = 0;
  c->fallback_periods = c->clean_periods = c->skipped_periods = c->sliver_periods = 0;
  std::memset(c->t_clean, 0, sizeof(c->t_clean));
  std::memset(c->t_fallback, 0, sizeof(c->t_fallback));
  std::memset(c->t_skipped, 0, sizeof(c->t_skipped));
  std::memset(c->t_sliver, 0, sizeof(c->t_sliver));
  std::memset(c->t_model, 0, sizeof(c->t_model));
  std::memset(c->t_moved, 0, sizeof(c->t_moved));
  c->cad_calls = 0;
  std::memset(c->t_delivered, 0, sizeof(c->t_delivered));
  std::memset(c->t_first_ns, 0, sizeof(c->t_first_ns));
  std::memset(c->t_last_ns, 0, sizeof(c->t_last_ns));
  c->align_samples = c->align_close = c->align_long = c->align_short = c->align_denied = 0;
  c->attr_harvested = c->attr_ticks_sum = c->attr_ticks_max = 0;
  c->attr_lag_sum_ns = 0;
  c->ts_gap_sum = 0;
  c->ts_gaps = 0;
  return 0;
}

// Sampler policy: budget % (token bucket over every hardware sample, 0: no
// budget), switch-aligned samples (0/1), calibrated model fallback (0/1); -1
// keeps a setting.  Returns 0.
int gpbs_gpu_hwc_sampler(void* p, int budget_pct, int align, int fallback) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  if (budget_pct >= 0) c->hwc_budget_pct = std::min(100, budget_pct);
  if (align >= 0) c->hwc_align = align != 0;
  if (fallback >= 0) c->model_fallback = fallback != 0;
  c->hwc_tokens = c->hwc_bucket;
  return 0;
}

// Switch-aligned sampling parameters (< 0 keeps): drain guard between a
// publish and its sample (us), the tenure length that opens a window at
// every switch (us), and how old a tenant's last clean window must be before
// the calibrated fallback stands in (us).  out8 (optional): aligned samples,
// of which closing a window / opening a long one / opening a short pair,
// switch samples denied by the budget, mean sample gap over intervals with a
// switch (ns, the time-shared cadence), clean-window tenant periods, skipped
// ones.
// Measurement-tenure requests the sampler made since the last hwc reset.
uint64_t gpbs_gpu_hwc_measure_reqs(void* p) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return 0;
  std::lock_guard<std::mutex> g(c->snap_mu);
  return c->measure_reqs;
}

int gpbs_gpu_hwc_align(void* p, int guard_us, int long_us, int stale_us, uint64_t* out8) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  if (guard_us >= 0) c->hwc_guard_us = guard_us;
  if (long_us >= 0) c->hwc_long_us = long_us;
  if (stale_us >= 0) c->hwc_stale_us = stale_us;
  if (out8) {
    out8[0] = c->align_samples;
    out8[1] = c->align_close;
    out8[2] = c->align_long;
    out8[3] = c->align_short;
    out8[4] = c->align_denied;
    out8[5] = c->ts_gaps ? (uint64_t)(c->ts_gap_sum / (int64_t)c->ts_gaps) : 0;
    out8[6] = c->clean_periods;
    out8[7] = c->skipped_periods;
  }
  return c->hwc_align;
}

// One tenant's metric periods since the last hwc reset: out4 = clean window,
// calibrated fallback, skipped (no clean window, not stale or uncalibrated),
// sliver (the edge of another tenure); out_cal4 (optional) its current
// hardware/model ratio per counter.
int gpbs_gpu_hwc_tenant_periods(void* p, int t, uint64_t* out4, double* out_cal4) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c || t < 0 || t >= kMaxTenants) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  if (out4) {
    out4[0] = c->t_clean[t];
    out4[1] = c->t_fallback[t];
    out4[2] = c->t_skipped[t];
    out4[3] = c->t_sliver[t];
  }
  if (out_cal4)
    for (int k = 0; k < kNumPmc; ++k) out_cal4[k] = c->cal[t][k];
  return 0;
}

// Debug: the cadence ring (tick time, tenants 1 and 2 instruction sums) of
// the last min(n, 512) ticks, oldest first; returns the count.
int gpbs_gpu_cadence_ring(void* p, int64_t* out, int n) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c || !out) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  const int have = (int)std::min<uint64_t>(c->cad_calls, 512);
  const int k = std::min(n, have);
  for (int i = 0; i < k; ++i) {
    const int64_t* d = c->cad_dbg[(c->cad_calls - k + i) % 512];
    out[3 * i] = d[0];
    out[3 * i + 1] = d[1];
    out[3 * i + 2] = d[2];
  }
  return k;
}

// Freshness probe of the host-readable counter block (tools): `n` reads of
// tenant t's instruction counter `gap_us` apart, through the BAR (mode 0) or
// a device-to-host copy (mode 1); returns how many reads saw a new value.
int gpbs_gpu_block_probe(void* p, int t, int n, int gap_us, int mode, int64_t* last) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c || t < 0 || t >= kMaxTenants || n <= 0) return -22;
  if (mode == 0 && !c->cnt_bar) return -95;
  u64 row[kXcds * kNumPmc];
  u64 prev = 0;
  int changed = 0;
  for (int i = 0; i < n; ++i) {
    if (mode == 0) {
      bar_read(c->d_cnt + (size_t)t * kXcds * kNumPmc, row, sizeof(row));
    } else if (hipMemcpy(row, c->d_cnt + (size_t)t * kXcds * kNumPmc, sizeof(row), hipMemcpyDeviceToHost) != hipSuccess) {
      return -5;
    }
    u64 v = 0;
    for (int x = 0; x < kXcds; ++x) v += row[x * kNumPmc];
    if (i && v != prev) ++changed;
    prev = v;
    const int64_t t0 = mono_ns();
    while (mono_ns() - t0 < (int64_t)gap_us * 1000) {
    }
  }
  if (last) *last = (int64_t)prev;
  return changed;
}

// Metric cadence of a tenant since the last hwc reset (round 6): out4 =
// metric periods delivered from the calibrated model (1 ms ticks), periods
// that delivered anything, the mean ns between delivering periods (0: fewer
// than two), whether the 1 ms cadence is live (host-readable block), the
// ticks its modeled counters moved, and the cadence ticks so far (out6).
int gpbs_gpu_hwc_tenant_cadence(void* p, int t, int64_t* out4) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c || t < 0 || t >= kMaxTenants || !out4) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  out4[0] = (int64_t)c->t_model[t];
  out4[1] = (int64_t)c->t_delivered[t];
  out4[2] = c->t_delivered[t] > 1 ? (c->t_last_ns[t] - c->t_first_ns[t]) / (int64_t)(c->t_delivered[t] - 1) : 0;
  out4[3] = c->model_cadence && c->cnt_bar;
  out4[4] = (int64_t)c->t_moved[t];
  out4[5] = (int64_t)c->cad_calls;
  return 0;
}

// Sample budget and model-fallback statistics: out[0] budget %, [1] burst
// ticks denied a token, [2] tenant-periods that reported calibrated modeled
// deltas (no clean window), [3] tenant-periods with a clean hardware window,
// [4] switch-aligned samples on (0/1), [5] model fallback on (0/1).
int gpbs_gpu_hwc_budget_stats(void* p, uint64_t* out5) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c || !out5) return -22;
  out5[5] = (uint64_t)c->model_fallback;
  std::lock_guard<std::mutex> g(c->snap_mu);
  out5[0] = (uint64_t)c->hwc_budget_pct;
  out5[1] = c->hwc_denied;
  out5[2] = c->fallback_periods;
  out5[3] = c->clean_periods;
  out5[4] = (uint64_t)c->hwc_align;
  return 0;
}

// Sampler cadence: fast and steady-state periods (us, < 0 leaves them), and
// *slow_samples = samples taken at the steady-state period since the last
// hwc reset.
// Returns the previous slow (back-off) period in us.
int gpbs_gpu_hwc_period(void* p, int fast_us, int slow_us, uint64_t* slow_samples) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  const int old = c->hwc_slow_us;
  if (fast_us >= 0) c->hwc_period_us = std::max(100, fast_us);
  if (slow_us >= 0) c->hwc_slow_us = slow_us;
  if (slow_samples) *slow_samples = c->hwc_slow_samples;
  return old;
}

// Burst statistics since the last hwc reset: triggers (owner changes and
// modeled phase changes) and hardware samples taken in bursts.
int gpbs_gpu_hwc_bursts(void* p, uint64_t* triggers, uint64_t* burst_samples) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  std::lock_guard<std::mutex> g(c->snap_mu);
  if (triggers) *triggers = c->hwc_triggers.load();
  if (burst_samples) *burst_samples = c->hwc_burst_samples;
  return c->hwc_burst_ms;
}

// Duty-cycle cap (percent, < 0 leaves it; 0 off); *mean_period_ns = mean
// sampler period since the last hwc reset.  Returns the old cap.
int gpbs_gpu_hwc_duty(void* p, int pct, uint64_t* mean_period_ns) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  const int old = c->hwc_duty_pct;
  if (pct >= 0) c->hwc_duty_pct = std::min(pct, 100);
  if (mean_period_ns) {
    std::lock_guard<std::mutex> g(c->snap_mu);
    *mean_period_ns = c->hwc_samples ? (uint64_t)(c->hwc_period_sum_ns / (int64_t)c->hwc_samples) : 0;
  }
  return old;
}

// SE-exclusive partitions: the nctx (= 4) partitions of an XCD are its shader
// engines; gated tenant kernels run only on SEs their tenant owns.
// Class-share mode on/off (default off; param share).
// Returns the previous setting; *share_ns (optional) = cumulative time in
// class-share mode since the last hwc reset.
int gpbs_gpu_set_share(void* p, int on, int64_t* share_ns) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  const int old = c->share_enable;
  if (on >= 0) {
    c->share_enable = on ? 1 : 0;
    if (!on) c->share.store(0, std::memory_order_release);
  }
  if (share_ns) {
    std::lock_guard<std::mutex> g(c->snap_mu);
    *share_ns = c->snap_share - c->share_base;
  }
  return old;
}

extern "C" int gpbs_hip_masked_pool_prealloc(int device, int* out, int max);
int gpbs_gpu_set_se_mode(void* p, int on) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  // SE mode launches on the process's CU-masked queue pool: make its burst
  // now, before the runners run.  Creating a hardware queue remaps the
  // process's runlist, which preempts every queue it has: the lazy burst at
  // the first SE-exclusive relayout froze ALL runners for ~100 ms
  // (profiles/r6/phase_debug_summary.txt).  A pool made earlier (the bench's
  // pipe pre-flight) is kept.  on == 2: SE mode without the pool -- a
  // process that launches no tenant kernel (gpbsd: its tenants are other
  // processes) must not hold ten idle hardware queues.
  if (on == 1 && gpbs_hip_masked_pool_prealloc(c->device, nullptr, 0) < 0) return -12;
  __atomic_store_n(&c->se_mode, on ? 1 : 0, __ATOMIC_RELEASE);
  if (!on) c->share.store(0, std::memory_order_release);  // class sharing exists only over SE partitions
  return 0;
}

// Latency-class runners (priority > 0) launch their kernels with raised wave
// issue priority while a gated policy is active.
// Latency-request hold (GATE_HOLD) on/off; returns the previous setting.
// *raises (optional): times the hold word was raised since the context began.
int gpbs_gpu_set_hold(void* p, int on, uint64_t* raises) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  const int old = c->hold_enable;
  if (on >= 0) {
    __atomic_store_n(&c->hold_enable, on ? 1 : 0, __ATOMIC_RELEASE);
    if (!on) {
      std::lock_guard<std::mutex> g(c->hold_mu);
      c->holds = 0;
      c->hold_gen++;  // raises still held by runners belong to the old generation
      set_hold(c, 0);
    }
  }
  if (raises) *raises = c->hold_raises.load();
  return old;
}

// Test hook: raise (1) or clear (0) the hold word directly.
int gpbs_gpu_force_hold(void* p, int v) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  std::lock_guard<std::mutex> g(c->hold_mu);
  set_hold(c, v ? 1u : 0u);
  return 0;
}

// Latency lane (see GpuCtx::lat_half): -1 off, 0 / 1 the class half.
int gpbs_gpu_set_lat_half(void* p, int half) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c || half < -1 || half > 1) return -22;
  __atomic_store_n(&c->lat_half, half, __ATOMIC_RELEASE);
  return 0;
}

int gpbs_gpu_set_waveprio(void* p, int on) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  __atomic_store_n(&c->waveprio, on ? 1 : 0, __ATOMIC_RELEASE);
  return 0;
}

int gpbs_gpu_set_spatial(void* p, int on) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  __atomic_store_n(&c->spatial, on ? 1 : 0, __ATOMIC_RELEASE);
  return 0;
}

int gpbs_gpu_set_table_mode(void* p, int mode) {
  GpuCtx* c = (GpuCtx*)p;
  std::lock_guard<std::mutex> g(c->mu);
  if (mode == 2) {
    if (!c->b_table) {
      hipSetDevice(c->device);
      c->b_table = bar_alloc(c->device);
      if (!c->b_table) return -95;  // no host-accessible fine-grained VRAM pool on this system
    }
    {
      std::lock_guard<std::mutex> hg(c->hold_mu);
      bar_sync(c->b_table, c->h_table);
    }
    __atomic_store_n(&c->table_mode, 2, __ATOMIC_RELEASE);
    return 0;
  }
  if (mode == 1) {
    if (hipMemcpyAsync(c->d_table, c->h_table, sizeof(PartTable), hipMemcpyHostToDevice, c->sched_stream) !=
            hipSuccess ||
        hipStreamSynchronize(c->sched_stream) != hipSuccess)
      return -5;
  }
  __atomic_store_n(&c->table_mode, mode == 1 ? 1 : 0, __ATOMIC_RELEASE);
  return 0;
}

void* gpbs_gpu_table(void* p) {
  GpuCtx* c = (GpuCtx*)p;
  return c->table_mode == 1 ? (void*)c->d_table : c->table_mode == 2 ? (void*)c->b_table : (void*)c->h_table;
}
int gpbs_gpu_table_mode(void* p) { return ((GpuCtx*)p)->table_mode; }
void* gpbs_gpu_counters(void* p) { return ((GpuCtx*)p)->d_cnt; }

// owners: [kXcds * kCtx] entries (kCtx = 4), (xcd, context) major, -1 = idle.
int gpbs_gpu_set_owners(void* p, const int* owners) {
  GpuCtx* c = (GpuCtx*)p;
  {
    std::lock_guard<std::mutex> g(c->mu);
    for (int x = 0; x < kXcds * kCtx; ++x) c->pending[x] = owners[x] >= 0 ? (u32)owners[x] : kNoOwner;
    publish_locked(c);
  }
  c->cv.notify_all();
  return 0;
}

int gpbs_gpu_get_owners(void* p, int* owners) {
  GpuCtx* c = (GpuCtx*)p;
  for (int x = 0; x < kXcds * kCtx; ++x) {
    u32 o = __atomic_load_n(&c->h_table->owner[x], __ATOMIC_ACQUIRE);
    if (o != kNoOwner) o &= kOwnerMask;
    owners[x] = o == kNoOwner ? -1 : (int)o;
  }
  return (int)c->h_table->epoch;
}

// Cumulative counters of a tenant summed over XCDs (synchronous; tests/tools).
int gpbs_gpu_read_counters(void* p, int tenant, uint64_t* out4, uint64_t* per_xcd32) {
  GpuCtx* c = (GpuCtx*)p;
  if (tenant < 0 || tenant >= kMaxTenants) return -22;
  u64 buf[kXcds * kNumPmc];
  if (c->cnt_bar) {
    HIPCHECK(hipDeviceSynchronize());  // finished kernels' counts have landed
    bar_read(c->d_cnt + (size_t)tenant * kXcds * kNumPmc, buf, sizeof(buf));
  } else {
    HIPCHECK(hipMemcpy(buf, c->d_cnt + (size_t)tenant * kXcds * kNumPmc, sizeof(buf), hipMemcpyDeviceToHost));
  }
  for (int i = 0; i < 4; ++i) {
    out4[i] = 0;
    for (int x = 0; x < kXcds; ++x) out4[i] += buf[x * 4 + i];
  }
  if (per_xcd32) std::memcpy(per_xcd32, buf, sizeof(buf));
  return 0;
}

// ns tenant `t` held context c (summed over XCDs), out[kCtx]; reset when clear != 0.
int gpbs_gpu_ownership(void* p, int t, int64_t* out2, int clear) {
  GpuCtx* c = (GpuCtx*)p;
  if (t < 0 || t >= kMaxTenants) return -22;
  std::lock_guard<std::mutex> g(c->mu);
  std::vector<int64_t> cum((size_t)kMaxTenants * kXcds * kCtx);
  own_snapshot_locked(c, cum.data());  // includes the interval since the last table change
  const int64_t* ct = cum.data() + (size_t)t * kXcds * kCtx;
  for (int k = 0; k < kCtx; ++k) {
    out2[k] = 0;
    for (int x = 0; x < kXcds; ++x) out2[k] += ct[x * kCtx + k] - c->own_base[t][x * kCtx + k];
  }
  if (clear) std::memcpy(c->own_base[t], ct, sizeof(c->own_base[t]));
  return 0;
}

// Device adapt: calls, results not back within the poll budget (host
// fallback that period), calls that found the previous launch still running.
int gpbs_gpu_adapt_stats(void* p, uint64_t* calls, uint64_t* late, uint64_t* busy) {
  GpuCtx* c = (GpuCtx*)p;
  if (!c) return -22;
  if (calls) *calls = c->adapt_calls + c->async_launches;
  if (late) *late = c->adapt_late + c->async_late;
  if (busy) *busy = c->adapt_busy + c->async_busy;
  return 0;
}

// Process-wide CU-masked queue pool: out[0] masked streams ever created,
// out[1] currently free (the rest are held by runners), out[2] acquires that
// had to share another layout's queue (over the budget: those layouts ran
// serialised), out[3] most queues held at once since the last reset, out[4]
// acquires that had to run on a pipe another class half's queue was using.  Every
// created one is a hardware queue this process keeps.  reset: restart the
// high-water mark at the number held now.
int gpbs_gpu_masked_pool(uint64_t* out5, int reset) {
  MaskedPoolCore& P = masked_pool();
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(P.mu);
  if (reset) P.held_max = P.held_locked(dev);
  if (!out5) return 0;
  out5[0] = P.created;
  uint64_t idle = 0;
  for (auto& e : P.ents) idle += e.refs == 0;
  out5[1] = idle;
  out5[2] = P.cross_key_shares;
  out5[3] = (uint64_t)P.held_max;
  out5[4] = P.pipe_shared_other;
  return 0;
}

// Host check of the masked-queue pool policy: fake queue handles,
// no HIP call.  Returns 0 or the number of the first failed check.
// Bench pre-flight: create this process's masked-queue
// burst now (normally at first use) -- after RCCL has made its own queues --
// and report it: returns the queues the pool holds on `device`, out[i] =
// pipe | half << 8 of pool queue i (the burst-relative pipe and the class
// half of its CU mask), max entries.  The caller compares the KFD queue ids
// the process gained around this call with the burst (one contiguous run).
int gpbs_hip_masked_pool_prealloc(int device, int* out, int max) {
  if (hipSetDevice(device) != hipSuccess) return -19;
  uint32_t mc[8], mm[8];
  half_mask(0, mc);
  half_mask(1, mm);
  const uint32_t* masks[2] = {mc, mm};
  auto create = [](const uint32_t* m) -> hipStream_t {
    hipStream_t s = nullptr;
    return hipExtStreamCreateWithCUMask(&s, 8, const_cast<uint32_t*>(m)) == hipSuccess ? s : nullptr;
  };
  MaskedPoolCore& P = masked_pool();
  if (P.prealloc(device, masks, kPlan, kPlanLen, create) < 0) return -12;
  std::lock_guard<std::mutex> g(P.mu);
  int n = 0;
  for (const auto& e : P.ents)
    if (e.device == device) {
      if (out && n < max) out[n] = e.pipe | ((std::memcmp(e.m, mm, sizeof(mm)) == 0 ? 1 : 0) << 8);
      ++n;
    }
  return n;
}

int gpbs_hip_masked_pool_selftest(void) {
  MaskedPoolCore P;
  uintptr_t next = 0x1000;
  auto mk = [&](const uint32_t*) -> hipStream_t { return (hipStream_t)(next += 0x10); };
  uint32_t mc[8], mm[8];
  for (int w = 0; w < 8; ++w) mc[w] = 0x33333333u, mm[w] = 0xCCCCCCCCu;
  // 1. co-sharers of one layout share one queue
  hipStream_t a = P.acquire(0, mc, 0x11, mk), b = P.acquire(0, mc, 0x11, mk);
  if (!a || a != b || P.created != 1) return 1;
  // 2. concurrent layouts on one mask get their own queues (no cap below the budget)
  hipStream_t c = P.acquire(0, mc, 0x22, mk), d = P.acquire(0, mc, 0x44, mk), e = P.acquire(0, mc, 0x88, mk);
  if (c == a || d == a || e == a || c == d || d == e || c == e || P.created != 4 || P.cross_key_shares) return 2;
  // 3. an exclusive acquire never gets a queue held under another key
  hipStream_t x = P.acquire(0, mc, 0, mk);
  if (x == a || x == c || x == d || x == e || P.created != 5) return 3;
  // 4. a released queue is re-keyed before a new one is created; refs drop to zero first
  P.release(c);
  hipStream_t f = P.acquire(0, mc, 0x99, mk);
  if (f != c || P.created != 5) return 4;
  P.release(a);
  hipStream_t g2 = P.acquire(0, mc, 0x55, mk);  // a still held once (b): not idle
  if (g2 == a || P.created != 6) return 5;
  // 5. another mask / device never shares
  hipStream_t h = P.acquire(0, mm, 0x11, mk), i = P.acquire(1, mc, 0x11, mk);
  if (h == a || i == a || h == i || P.created != 8) return 6;
  // 6. past the budget a new layout shares the least-held keyed queue, counted
  for (int k = 0; (int)P.created < kMaskedBudget + 1; ++k) P.acquire(0, mm, 0x1000u + k, mk);
  const uint64_t cr = P.created;
  hipStream_t j = P.acquire(0, mc, 0x7777, mk);
  if (P.created != cr || P.cross_key_shares != 1 || !j) return 7;
  // 7. an exclusive acquire past the budget still gets a queue of its own
  hipStream_t k2 = P.acquire(0, mc, 0, mk);
  for (auto& en : P.ents)
    if (en.s == k2 && en.refs != 1) return 8;
  if (P.held_max < kMaskedBudget) return 9;
  // 8. pipes: queues created consecutively sit on consecutive pipes; a memory
  //    layout next to a running compute queue avoids the compute queue's pipe
  MaskedPoolCore Q;
  hipStream_t c0 = Q.acquire(0, mc, 0x1, mk);  // index 0: pipe 0
  hipStream_t m1 = Q.acquire(0, mm, 0x2, mk), m2 = Q.acquire(0, mm, 0x3, mk), m3 = Q.acquire(0, mm, 0x4, mk);
  hipStream_t m4 = Q.acquire(0, mm, 0x5, mk);  // index 4: pipe 0, the compute queue's
  if (Q.pipe_of(c0) != 0 || Q.pipe_of(m1) != 1 || Q.pipe_of(m4) != 0 || Q.pipe_shared_other != 1) return 10;
  Q.release(m1);
  Q.release(m4);
  hipStream_t n1 = Q.acquire(0, mm, 0x9, mk);  // idle on pipes 1 and 0: takes pipe 1
  if (n1 != m1) return 11;
  hipStream_t n2 = Q.acquire(0, mm, 0xA, mk);  // idle m4 shares the compute pipe: a new one (index 5, pipe 1) is cheaper
  if (n2 == m4 || Q.pipe_of(n2) != 1 || Q.created != 6) return 12;
  (void)m2;
  (void)m3;
  // 9. the burst: the plan's queues on consecutive pipes, compute alone on
  //    pipe 0; a compute layout and three memory layouts never share a pipe
  MaskedPoolCore R;
  const uint32_t* masks[2] = {mc, mm};
  if (R.prealloc(0, masks, kPlan, kPlanLen, mk) != kPlanLen || R.created != (uint64_t)kPlanLen) return 13;
  if (R.prealloc(0, masks, kPlan, kPlanLen, mk) != 0) return 14;
  hipStream_t rc = R.acquire(0, mc, 0x1, mk);
  hipStream_t r1 = R.acquire(0, mm, 0x2, mk), r2 = R.acquire(0, mm, 0x4, mk), r3 = R.acquire(0, mm, 0x8, mk);
  if (R.pipe_of(rc) != 0 || R.pipe_of(r1) == 0 || R.pipe_of(r2) == 0 || R.pipe_of(r3) == 0) return 15;
  if (R.pipe_of(r1) == R.pipe_of(r2) || R.pipe_of(r2) == R.pipe_of(r3) || R.pipe_of(r1) == R.pipe_of(r3)) return 16;
  // the 8mix static split (3 compute, 4 memory, the exclusive lane): no
  // creation past the burst, no cross-key share, no memory queue on pipe 0
  hipStream_t rc2 = R.acquire(0, mc, 0x10, mk), rc3 = R.acquire(0, mc, 0x20, mk);
  hipStream_t r4 = R.acquire(0, mm, 0x40, mk), lane = R.acquire(0, mm, 0, mk);
  if (R.created != (uint64_t)kPlanLen || R.cross_key_shares || R.pipe_shared_other) return 17;
  if (R.pipe_of(rc2) != 0 || R.pipe_of(rc3) != 0 || R.pipe_of(r4) == 0 || R.pipe_of(lane) == 0) return 18;
  // 10. dispatch-rate weights: four memory layouts on three memory pipes --
  //     two streams, a launch-bound tenant, a latency tenant -- the
  //     launch-bound one never shares a pipe with a stream, in any order
  const double loads[4] = {2500, 2500, 20000, 500};
  const int orders[4][4] = {{0, 1, 2, 3}, {2, 0, 1, 3}, {3, 0, 1, 2}, {0, 3, 2, 1}};
  for (const auto& ord : orders) {
    MaskedPoolCore W;
    if (W.prealloc(0, masks, kPlan, kPlanLen, mk) != kPlanLen) return 19;
    W.acquire(0, mc, 0x1, mk, 100000);  // the compute layout on pipe 0
    hipStream_t q4[4];
    for (int i : ord) q4[i] = W.acquire(0, mm, 0x10u << i, mk, loads[i]);
    const int pb = W.pipe_of(q4[2]);
    if (pb == 0 || pb == W.pipe_of(q4[0]) || pb == W.pipe_of(q4[1])) return 20;
    W.release(q4[2], loads[2]);
    for (auto& en : W.ents)
      if (en.s == q4[2] && (en.refs || en.load != 0)) return 21;
  }
  return 0;
}

int gpbs_gpu_stats(void* p, uint64_t* out4) {
  GpuCtx* c = (GpuCtx*)p;
  out4[0] = c->switches.load();
  out4[1] = c->flushes.load();
  out4[2] = c->metric_calls.load();
  out4[3] = (uint64_t)c->metric_ns;
  return 0;
}

// CU-masked stream for foreign kernels (torch/hipBLASLt/RCCL tenants): a
// stream whose hardware queue only dispatches to the CUs in `cu_mask`
// (nwords x 32 bits, hipExtStreamCreateWithCUMask).
// End-to-end actuation latency (perf-regression microbench): the time from
// the scheduler's publish of a new assignment to EVERY workgroup of a probe
// grid (nwg one-wave workgroups spread over all XCDs / shader engines)
// having observed the new epoch, per iteration, in out_ns[iters].  Uses the
// context's own table in its current mode (host: one release store;
// device: + the k_partition_switch launch on the scheduler stream).  Only
// on a context with no engine attached.  Returns iterations measured or <0.
int gpbs_gpu_switch_latency(void* p, int iters, int nwg, int64_t* out_ns) {
  GpuCtx* c = (GpuCtx*)p;
  if (c->engine || iters <= 0 || nwg <= 0 || nwg > 4096) return -22;
  hipSetDevice(c->device);
  constexpr u32 kStop = 0xFFFFFFF0u;
  u32* acks = nullptr;
  if (hipHostMalloc((void**)&acks, sizeof(u32) * nwg, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
    return -12;
  for (int i = 0; i < nwg; ++i) __atomic_store_n(&acks[i], 0xFFFFFFFEu, __ATOMIC_RELAXED);
  hipStream_t ps = nullptr;
  hipStreamCreateWithFlags(&ps, hipStreamNonBlocking);
  const int tm = c->table_mode, dev = tm != 0;
  const void* tab = tm == 1 ? (const void*)c->d_table : tm == 2 ? (const void*)c->b_table : (const void*)c->h_table;
  // every wave exits after 20 s of device wall clock even if the host died
  int rc = gpbs_hip_switch_probe(tab, dev, acks, nwg, kStop, 20ull * 100000000ull, ps);
  // e == 0xFFFFFFFE: every wave has acknowledged some epoch (grid resident)
  auto all_acked = [&](u32 e, int64_t timeout_ns) {
    const int64_t t_end = mono_ns() + timeout_ns;
    for (;;) {
      bool ok = true;
      for (int i = 0; i < nwg && ok; ++i) {
        const u32 a = __atomic_load_n(&acks[i], __ATOMIC_ACQUIRE);
        ok = e == 0xFFFFFFFEu ? a != e : a == e;
      }
      if (ok) return true;
      if (mono_ns() > t_end) return false;
    }
  };
  int done = 0;
  if (rc == 0 && all_acked(0xFFFFFFFEu, 2000000000LL)) {
    for (int it = 0; it < iters; ++it) {
      const int64_t t0 = mono_ns();
      u32 e;
      {
        std::lock_guard<std::mutex> g(c->mu);
        for (int x = 0; x < kXcds * kCtx; ++x) c->pending[x] = (u32)((it + x) & 1);
        publish_locked(c);
        e = c->epoch;
      }
      if (!all_acked(e, 100000000LL)) {
        rc = -110;
        break;
      }
      out_ns[it] = mono_ns() - t0;
      done++;
    }
  } else if (rc == 0) {
    rc = -110;  // the probe grid never became resident
  }
  // stop epoch, then drain the probe grid (bounded by its own wall-clock exit)
  __atomic_store_n(&c->h_table->epoch, kStop, __ATOMIC_RELEASE);
  if (tm == 1) gpbs_hip_partition_switch(c->d_table, kStop, c->pending, c->sched_stream);
  if (tm == 2) bar_write(c->b_table, c->h_table->owner, kStop);
  const int64_t t_end = mono_ns() + 25000000000LL;
  while (hipStreamQuery(ps) == hipErrorNotReady && mono_ns() < t_end)
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  hipStreamSynchronize(ps);
  __atomic_store_n(&c->h_table->epoch, c->epoch, __ATOMIC_RELEASE);
  if (tm == 1) gpbs_hip_partition_switch(c->d_table, c->epoch, c->pending, c->sched_stream);
  if (tm == 2) bar_write(c->b_table, c->h_table->owner, c->epoch);
  hipStreamSynchronize(c->sched_stream);
  hipStreamDestroy(ps);
  hipHostFree(acks);
  return rc < 0 ? rc : done;
}

// roctx helpers for the Python side (gang epochs, bench policy windows).
int gpbs_roctx_push(const char* m) { return roctxRangePushA(m); }
int gpbs_roctx_pop(void) { return roctxRangePop(); }
void gpbs_roctx_mark(const char* m) { roctxMarkA(m); }

void* gpbs_gpu_cumask_stream(int device, const uint32_t* cu_mask, int nwords, int priority) {
  hipSetDevice(device);
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, cu_mask) != hipSuccess) return nullptr;
  (void)priority;
  return (void*)s;
}

int gpbs_gpu_stream_destroy(void* s) { return hipStreamDestroy((hipStream_t)s) == hipSuccess ? 0 : -5; }

void* gpbs_runner_create(void* ctx, const gpbs_runner_cfg_t* cfg) {
  GpuCtx* c = (GpuCtx*)ctx;
  if (!c || !cfg || cfg->tenant < 0 || cfg->tenant >= kMaxTenants) return nullptr;
  if (cfg->kind == K_GEMM && (cfg->M % 128 || cfg->N % 128 || cfg->K % 64)) return nullptr;
  if ((cfg->kind == K_STREAM || cfg->kind == K_REDUCE) && (cfg->bytes % 16 || cfg->chunk_bytes <= 0 || cfg->chunk_bytes % 16))
    return nullptr;
  if (cfg->kind == K_GEMV && cfg->K % 512) return nullptr;
  if (cfg->kind == K_ALLREDUCE &&
      (!cfg->a || cfg->M < 1 || cfg->M > kCollMax || cfg->N < 0 || cfg->N >= cfg->M || cfg->bytes % (16ull * cfg->M) ||
       cfg->chunk_bytes <= 0 || cfg->chunk_bytes % 16))
    return nullptr;
  if (cfg->alt_kind == K_GEMM && (cfg->alt_M % 128 || cfg->alt_N % 128 || cfg->alt_K % 64)) return nullptr;
  if ((cfg->alt_kind == K_STREAM || cfg->alt_kind == K_REDUCE) &&
      (cfg->alt_bytes % 16 || cfg->alt_chunk_bytes <= 0 || cfg->alt_chunk_bytes % 16))
    return nullptr;
  if (cfg->alt_kind == K_GEMV && cfg->alt_K % 512) return nullptr;
  if (cfg->alt_kind < 0 || cfg->alt_kind > K_GEMV) return nullptr;
  hipSetDevice(c->device);
  for (int have = c->cnt_rows.load(); have < cfg->tenant + 1 && !c->cnt_rows.compare_exchange_weak(have, cfg->tenant + 1);) {
  }
  auto* r = new Runner;
  r->ctx = c;
  r->cfg = *cfg;
  if (r->cfg.depth <= 0) r->cfg.depth = 2;
  if (r->cfg.depth > 8) r->cfg.depth = 8;
  r->nq = r->cfg.depth + 1;
  int lo = 0, hi = 0;
  hipDeviceGetStreamPriorityRange(&lo, &hi);
  bool ok = hipStreamCreateWithPriority(&r->stream, hipStreamNonBlocking, cfg->priority ? hi : lo) == hipSuccess;
  ok = ok && hipMalloc((void**)&r->d_q, sizeof(WorkQueue) * r->nq) == hipSuccess;
  // zeroed once: a kernel that completes every unit leaves its queue zeroed
  // (finish()), so fresh launches need no memset on the tenant stream
  ok = ok && hipMemset(r->d_q, 0, sizeof(WorkQueue) * r->nq) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&r->h_status, sizeof(u32) * r->nq, hipHostMallocCoherent | hipHostMallocMapped) ==
                 hipSuccess;
  for (int i = 0; i < r->nq && ok; ++i) ok = hipEventCreateWithFlags(&r->ev[i], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    delete r;
    return nullptr;
  }
  r->th = std::thread([r] { r->loop(); });
  return r;
}

int gpbs_runner_submit(void* p, int units) {
  Runner* r = (Runner*)p;
  const int64_t t = mono_ns();
  {
    std::lock_guard<std::mutex> g(r->mu);
    r->pending += units;
    r->st.submitted += units;
    for (int i = 0; i < units; ++i) r->submit_times.push_back(t);
  }
  r->cv.notify_all();
  return 0;
}

// Block until every submitted unit has completed. Returns 0, or -110 on timeout.
int gpbs_runner_wait(void* p, int64_t timeout_ns) {
  Runner* r = (Runner*)p;
  std::unique_lock<std::mutex> lk(r->mu);
  auto pred = [&] { return (r->pending <= 0 && r->inflight <= 0) || r->stop; };
  if (timeout_ns <= 0) {
    r->idle_cv.wait(lk, pred);
    return r->err;
  }
  return r->idle_cv.wait_for(lk, std::chrono::nanoseconds(timeout_ns), pred) ? r->err : -110;
}

int gpbs_runner_stats(void* p, gpbs_runner_stats_t* out) {
  Runner* r = (Runner*)p;
  std::lock_guard<std::mutex> g(r->mu);
  *out = r->st;
  return 0;
}

// Which CU-masked queue of the process pool the runner launches on now
// (the pool index, stable for the process: entries are never removed; the
// latency lane's class-half queue if it has one), or -1 (its own stream).
// Diagnostics: which hardware queue -- and so which pipe -- a slow run used.
int gpbs_runner_queue(void* p) {
  Runner* r = (Runner*)p;
  hipStream_t s = r->key_stream ? r->key_stream : (r->se_stream[0] ? r->se_stream[0] : r->se_stream[1]);
  if (!s) return -1;
  MaskedPoolCore& P = masked_pool();
  std::lock_guard<std::mutex> g(P.mu);
  for (size_t i = 0; i < P.ents.size(); ++i)
    if (P.ents[i].s == s) return (int)i;
  return -1;
}

// Copy up to max latency samples (ns); returns count.
int gpbs_runner_latencies(void* p, int64_t* out, int max, int clear) {
  Runner* r = (Runner*)p;
  std::lock_guard<std::mutex> g(r->mu);
  if (!out) return (int)r->lats.size();
  int n = (int)std::min<size_t>(r->lats.size(), (size_t)max);
  std::memcpy(out, r->lats.data(), sizeof(int64_t) * n);
  if (clear) {
    r->lats.clear();
    r->st.lat_sum_ns = r->st.lat_max_ns = 0;
    r->st.lat_count = 0;
  }
  return n;
}

int gpbs_runner_reset_stats(void* p) {
  Runner* r = (Runner*)p;
  std::lock_guard<std::mutex> g(r->mu);
  const uint64_t sub = r->st.submitted - r->st.units_done;
  r->st = gpbs_runner_stats_t{};
  r->st.submitted = sub;
  r->lats.clear();
  return 0;
}

// Drop every submitted unit that has not been launched yet (units in flight
// complete); returns the number dropped.  Used to end a backlogged
// (steady-state) measurement window.
int64_t gpbs_runner_cancel(void* p) {
  Runner* r = (Runner*)p;
  std::lock_guard<std::mutex> g(r->mu);
  const int64_t n = r->pending;
  r->pending = 0;
  for (int64_t i = 0; i < n && !r->submit_times.empty(); ++i) r->submit_times.pop_back();
  r->st.submitted -= (uint64_t)n;
  if (r->inflight <= 0) r->idle_cv.notify_all();
  return n;
}

int gpbs_runner_set_gate(void* p, int gate) {
  Runner* r = (Runner*)p;
  std::lock_guard<std::mutex> g(r->mu);
  r->cfg.gate = gate;
  return 0;
}

int gpbs_runner_set_engine_wake(void* p, int on) {
  Runner* r = (Runner*)p;
  std::lock_guard<std::mutex> g(r->mu);
  r->cfg.engine_wake = on;
  return 0;
}

void* gpbs_runner_stream(void* p) { return ((Runner*)p)->stream; }

// Phase-changing tenant: fresh units use the alternate workload (1) or the
// primary one (0).  Returns the previous phase, -22 without an alternate.
int gpbs_runner_set_phase(void* p, int alt) {
  Runner* r = (Runner*)p;
  if (!r->cfg.alt_kind) return -22;
  return r->phase.exchange(alt ? 1 : 0, std::memory_order_acq_rel);
}

void gpbs_runner_destroy(void* p) {
  Runner* r = (Runner*)p;
  if (!r) return;
  {
    std::lock_guard<std::mutex> g(r->mu);
    r->stop = true;
  }
  r->cv.notify_all();
  r->ctx->cv.notify_all();
  if (r->th.joinable()) r->th.join();
  hipStreamSynchronize(r->stream);
  for (int i = 0; i < r->nq; ++i) hipEventDestroy(r->ev[i]);
  hipStreamDestroy(r->stream);
  for (int h = 0; h < 2; ++h) {  // masked streams go back to the process pool
    uint32_t m[8];
    if (r->half_stream[h]) {
      half_mask(h, m);
      masked_release(m, r->half_stream[h]);
    }
    if (r->se_stream[h]) {
      Runner::se_half_mask(h, m);
      masked_release(m, r->se_stream[h]);
    }
  }
  if (r->key_stream) masked_pool().release(r->key_stream, r->key_load);
  hipFree(r->d_q);
  hipHostFree(r->h_status);
  delete r;
}

// ---- all-reduce tenant buffers: one Coll per rank, peers over IPC ----------
void* gpbs_coll_create(int device, int rank, int world, unsigned long long bytes) {
  if (world < 1 || world > kCollMax || rank < 0 || rank >= world || bytes == 0 || bytes % (16ull * world)) return nullptr;
  if ((int)sizeof(CollDescHost) != gpbs_hip_coll_desc_size()) return nullptr;  // host / device layouts agree
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  auto* c = new Coll;
  c->device = device;
  c->rank = rank;
  c->world = world;
  c->bytes = bytes;
  // Flag words in UNCACHED device memory: they are written by other ranks
  // (over xGMI, or from another process on the same GPU) and polled by
  // workgroups on every XCD, and a coarse-grained line can sit stale in an
  // XCD's L2 (measured: a barrier polled a value the host read as updated for
  // 3 s until its timeout).
  bool ok = hipMalloc(&c->in, bytes) == hipSuccess && hipMalloc(&c->out, bytes) == hipSuccess &&
            hipExtMallocWithFlags((void**)&c->flags, 4096, hipDeviceMallocUncached) == hipSuccess &&
            hipMemset(c->flags, 0, 4096) == hipSuccess &&
            hipMemset(c->out, 0, bytes) == hipSuccess && hipMalloc(&c->d_desc, sizeof(CollDescHost)) == hipSuccess;
  if (!ok) {
    if (c->in) hipFree(c->in);
    if (c->out) hipFree(c->out);
    if (c->flags) hipFree(c->flags);
    delete c;
    return nullptr;
  }
  c->desc.rank = (u32)rank;
  c->desc.world = (u32)world;
  c->desc.n8 = bytes / 16;
  c->desc.in[rank] = c->in;
  c->desc.out[rank] = c->out;
  c->desc.flags[rank] = c->flags;
  return c;
}

// The three IPC handles (input, output, flags) of this rank's buffers, 3 x
// sizeof(hipIpcMemHandle_t) bytes into out.  Returns the byte count.
int gpbs_coll_export(void* p, void* out) {
  Coll* c = (Coll*)p;
  if (!c || !out) return -22;
  hipSetDevice(c->device);
  hipIpcMemHandle_t h[3];
  if (hipIpcGetMemHandle(&h[0], c->in) != hipSuccess || hipIpcGetMemHandle(&h[1], c->out) != hipSuccess ||
      hipIpcGetMemHandle(&h[2], c->flags) != hipSuccess)
    return -5;
  std::memcpy(out, h, sizeof(h));
  return (int)sizeof(h);
}

int gpbs_coll_handle_bytes(void) { return (int)(3 * sizeof(hipIpcMemHandle_t)); }

// Map peer `peer`'s buffers from its exported handles.
int gpbs_coll_open(void* p, int peer, const void* handles) {
  Coll* c = (Coll*)p;
  if (!c || !handles || peer < 0 || peer >= c->world || peer == c->rank) return -22;
  hipSetDevice(c->device);
  hipIpcMemHandle_t h[3];
  std::memcpy(h, handles, sizeof(h));
  for (int k = 0; k < 3; ++k) {
    if (c->peer[k][peer]) continue;
    if (hipIpcOpenMemHandle(&c->peer[k][peer], h[k], hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      c->peer[k][peer] = nullptr;
      return -5;
    }
  }
  c->desc.in[peer] = c->peer[0][peer];
  c->desc.out[peer] = c->peer[1][peer];
  c->desc.flags[peer] = (u32*)c->peer[2][peer];
  return 0;
}

// Every peer mapped: upload the descriptor the kernel reads.
int gpbs_coll_finalize(void* p) {
  Coll* c = (Coll*)p;
  if (!c) return -22;
  for (int r = 0; r < c->world; ++r)
    if (!c->desc.in[r] || !c->desc.out[r] || !c->desc.flags[r]) return -19;
  hipSetDevice(c->device);
  return hipMemcpy(c->d_desc, &c->desc, sizeof(c->desc), hipMemcpyHostToDevice) == hipSuccess ? 0 : -5;
}

// 0: input, 1: output, 2: flag words (this rank's device pointers); 3: the device descriptor.
void* gpbs_coll_buffer(void* p, int which) {
  Coll* c = (Coll*)p;
  if (!c) return nullptr;
  switch (which) {
    case 0: return c->in;
    case 1: return c->out;
    case 2: return c->flags;
    case 3: return c->d_desc;
  }
  return nullptr;
}

// Copy between a device buffer of the caller (a torch tensor) and this
// rank's input (0) / output (1) buffer; to_coll: 1 caller -> coll.  which 2:
// read this rank's flag words (diagnostics).
int gpbs_coll_copy(void* p, int which, void* dptr, unsigned long long bytes, int to_coll) {
  Coll* c = (Coll*)p;
  if (!c || !dptr || which < 0 || which > 2 || bytes > c->bytes || (which == 2 && (to_coll || bytes > 4096)))
    return -22;
  hipSetDevice(c->device);
  void* buf = which == 2 ? (void*)c->flags : which ? c->out : c->in;
  const hipError_t e = to_coll ? hipMemcpy(buf, dptr, bytes, hipMemcpyDeviceToDevice)
                               : hipMemcpy(dptr, buf, bytes, hipMemcpyDeviceToDevice);
  return e == hipSuccess ? 0 : -5;
}

// ---- gang epoch exchange over xGMI (coll_kernels.hip k_gang_exchange) ----
struct GangDescHost {
  long long* board[kCollMax];
  u32 rank, world, stride, nvals;
};

struct GangX {
  int device = 0, rank = 0, world = 1, nvals = 0;
  size_t board_bytes = 0;
  long long* board = nullptr;          // this rank's board (uncached VRAM)
  void* peer[kCollMax] = {};           // opened IPC mappings
  GangDescHost desc{};
  void* d_desc = nullptr;
  long long* h_vals = nullptr;         // pinned: this rank's values
  long long* h_out = nullptr;          // pinned: world x nvals rows
  u32* h_status = nullptr;             // pinned: 0 running, 1 yielded, 2 done
  hipStream_t stream = nullptr;
  uint64_t exchanges = 0, relaunches = 0, timeouts = 0;
};

void* gpbs_gangx_create(int device, int rank, int world, int nvals) {
  if (world < 1 || world > kCollMax || rank < 0 || rank >= world || nvals < 1 || nvals > 256) return nullptr;
  if ((int)sizeof(GangDescHost) != gpbs_hip_gang_desc_size()) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  auto* g = new GangX;
  g->device = device;
  g->rank = rank;
  g->world = world;
  g->nvals = nvals;
  const u32 stride = (u32)((nvals + 1 + 7) & ~7);  // 64-byte rows
  g->board_bytes = (size_t)2 * world * stride * sizeof(long long);
  bool ok = hipExtMallocWithFlags((void**)&g->board, g->board_bytes, hipDeviceMallocUncached) == hipSuccess &&
            hipMemset(g->board, 0, g->board_bytes) == hipSuccess &&
            hipMalloc(&g->d_desc, sizeof(GangDescHost)) == hipSuccess &&
            hipHostMalloc((void**)&g->h_vals, sizeof(long long) * nvals, hipHostMallocCoherent) == hipSuccess &&
            hipHostMalloc((void**)&g->h_out, sizeof(long long) * nvals * world, hipHostMallocCoherent) == hipSuccess &&
            hipHostMalloc((void**)&g->h_status, sizeof(u32), hipHostMallocCoherent) == hipSuccess &&
            hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) == hipSuccess &&
            hipDeviceSynchronize() == hipSuccess;
  if (!ok) {
    if (g->board) hipFree(g->board);
    if (g->d_desc) hipFree(g->d_desc);
    if (g->h_vals) hipHostFree(g->h_vals);
    if (g->h_out) hipHostFree(g->h_out);
    if (g->h_status) hipHostFree(g->h_status);
    delete g;
    return nullptr;
  }
  g->desc.rank = (u32)rank;
  g->desc.world = (u32)world;
  g->desc.stride = stride;
  g->desc.nvals = (u32)nvals;
  g->desc.board[rank] = g->board;
  return g;
}

int gpbs_gangx_handle_bytes(void) { return (int)sizeof(hipIpcMemHandle_t); }

int gpbs_gangx_export(void* p, void* out) {
  GangX* g = (GangX*)p;
  if (!g || !out) return -22;
  hipSetDevice(g->device);
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, g->board) != hipSuccess) return -5;
  std::memcpy(out, &h, sizeof(h));
  return (int)sizeof(h);
}

int gpbs_gangx_open(void* p, int peer, const void* handle) {
  GangX* g = (GangX*)p;
  if (!g || !handle || peer < 0 || peer >= g->world || peer == g->rank) return -22;
  hipSetDevice(g->device);
  if (!g->peer[peer]) {
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof(h));
    if (hipIpcOpenMemHandle(&g->peer[peer], h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      g->peer[peer] = nullptr;
      return -5;
    }
  }
  g->desc.board[peer] = (long long*)g->peer[peer];
  return 0;
}

int gpbs_gangx_finalize(void* p) {
  GangX* g = (GangX*)p;
  if (!g) return -22;
  for (int r = 0; r < g->world; ++r)
    if (!g->desc.board[r]) return -19;
  hipSetDevice(g->device);
  return hipMemcpy(g->d_desc, &g->desc, sizeof(g->desc), hipMemcpyHostToDevice) == hipSuccess ? 0 : -5;
}

// One exchange: this rank's n values in, every rank's rows out (world x
// nvals, rank order).  seq: 1, 2, ... (the same on every rank).  Returns 0,
// or -110 when deadline_ns (CLOCK_MONOTONIC) passed first -- the rank then
// treats the gang as failed (the caller degrades to local scheduling); a
// kernel still in flight leaves within its 200 us yield bound.
int gpbs_gangx_exchange(void* p, unsigned seq, const long long* vals, int n, long long* out, long long deadline_ns) {
  GangX* g = (GangX*)p;
  if (!g || !vals || !out || n < 0 || n > g->nvals || seq == 0) return -22;
  hipSetDevice(g->device);
  hipStreamSynchronize(g->stream);  // a yielded / abandoned launch has left
  for (int k = 0; k < g->nvals; ++k) g->h_vals[k] = k < n ? vals[k] : 0;
  constexpr unsigned long long kYieldTicks = 20000;  // 200 us of the 100 MHz wall clock
  for (;;) {
    __atomic_store_n(g->h_status, 0u, __ATOMIC_RELEASE);
    if (gpbs_hip_gang_exchange(g->d_desc, seq, g->h_vals, g->h_out, g->h_status, kYieldTicks, g->stream)) return -5;
    u32 st = 0;
    for (;;) {
      st = __atomic_load_n(g->h_status, __ATOMIC_ACQUIRE);
      if (st) break;
      if (mono_ns() > deadline_ns) {
        g->timeouts++;
        return -110;
      }
      std::this_thread::yield();
    }
    if (st == 2) break;
    g->relaunches++;
    hipStreamSynchronize(g->stream);
    if (mono_ns() > deadline_ns) {
      g->timeouts++;
      return -110;
    }
  }
  std::memcpy(out, g->h_out, sizeof(long long) * (size_t)g->nvals * g->world);
  g->exchanges++;
  return 0;
}

int gpbs_gangx_stats(void* p, uint64_t* out3) {
  GangX* g = (GangX*)p;
  if (!g || !out3) return -22;
  out3[0] = g->exchanges;
  out3[1] = g->relaunches;
  out3[2] = g->timeouts;
  return 0;
}

void gpbs_gangx_destroy(void* p) {
  GangX* g = (GangX*)p;
  if (!g) return;
  hipSetDevice(g->device);
  hipStreamSynchronize(g->stream);
  hipStreamDestroy(g->stream);
  for (int r = 0; r < kCollMax; ++r)
    if (g->peer[r]) hipIpcCloseMemHandle(g->peer[r]);
  hipFree(g->board);
  hipFree(g->d_desc);
  hipHostFree(g->h_vals);
  hipHostFree(g->h_out);
  hipHostFree(g->h_status);
  delete g;
}

void gpbs_coll_destroy(void* p) {
  Coll* c = (Coll*)p;
  if (!c) return;
  hipSetDevice(c->device);
  hipDeviceSynchronize();
  for (int k = 0; k < 3; ++k)
    for (int r = 0; r < kCollMax; ++r)
      if (c->peer[k][r]) hipIpcCloseMemHandle(c->peer[k][r]);
  hipFree(c->in);
  hipFree(c->out);
  hipFree(c->flags);
  hipFree(c->d_desc);
  delete c;
}

}  // extern "C"
