// Scheduler hot-path kernels (gfx950):
//   k_partition_switch : publishes a new XCD->tenant assignment (+epoch) into
//                        the device partition table (GPBS_TABLE=device mode).
//   k_counter_reduce   : per-tenant counter deltas.  One wave per tenant; lane
//                        = xcd*4 + counter; segmented sum across the 8 XCD
//                        lanes by DPP/shuffle; prev snapshot updated in place.
//                        (csched_dom_metric_update, X:xen/common/sched_credit.c:391-448)
//   k_adapt            : batched PBS phase detector / quantum update, one lane
//                        per tenant, same single-source integer code as the
//                        host engine (csrc/core/adapt_impl.h), bit-exact.
#include "common.hpp"
#include "../core/adapt_impl.h"
#include "../include/gpbs/gpbs.h"

namespace gpbs_hip {

struct Owners {
  u32 o[kXcds * kCtx];
};

// The scheduler's kernels run at top SIMD issue priority: they share CUs with
// the tenants' persistent waves, and their latency is the actuation latency.
__global__ void k_partition_switch(PartTable* t, u32 epoch, Owners ow) {
  __builtin_amdgcn_s_setprio(3);
  const int i = threadIdx.x;
  if (i < kXcds * kCtx) __hip_atomic_store(&t->owner[i], ow.o[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __syncthreads();
  if (i != 0) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(&t->epoch, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// cnt/prev: [kMaxTenants][kXcds][kNumPmc]; ids[n]; out[n][4] (host-mapped).
__global__ __launch_bounds__(64) void k_counter_reduce(u64* cnt, u64* prev, const int* ids, int n, u64* out) {
  __builtin_amdgcn_s_setprio(3);
  const int k = blockIdx.x;
  if (k >= n) return;
  const int lane = threadIdx.x;
  const int tid = ids[k];
  u64 d = 0;
  if (lane < kXcds * kNumPmc && tid >= 0 && tid < kMaxTenants) {
    const size_t off = (size_t)tid * kXcds * kNumPmc + lane;
    const u64 c = __hip_atomic_load(cnt + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const u64 p = prev[off];
    d = c >= p ? c - p : 0;  // Q5: counter reset -> no negative delta
    prev[off] = c;
  }
  // Sum the 8 XCD lanes of each counter (lane = xcd*4 + c): xor 4, 8, 16.
#pragma unroll
  for (int off = 4; off < kXcds * kNumPmc; off <<= 1) d += __shfl_xor(d, off, 64);
  if (lane < kNumPmc) out[(size_t)k * kNumPmc + lane] = d;
}

struct DevParams {
  u32 threshold, band_lo, band_hi, min_us, max_us, inc_us, dec_us, switch_boundary, ticks_per_tslice, spin_floor,
      scale, strict_ref, reserved;
};

__global__ __launch_bounds__(64) void k_adapt(gpbs_adapt_state_t* states, const u64* deltas, const u64* spin_sum,
                                             const u64* spin_cnt, int n, DevParams p, int* dirs) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  gpbs_adapt_state_t s = states[k];
  const int r = gpbs::impl::update(s, p, deltas[4 * k + 0], deltas[4 * k + 3], spin_sum[k], spin_cnt[k]);
  states[k] = s;
  if (dirs) dirs[k] = r;
}

}  // namespace gpbs_hip

using namespace gpbs_hip;

extern "C" {

// Switch-latency probe (perf-regression microbench, the analog of the perfctr
// init-time tests L:drivers/perfctr/x86_tests.c:181-245): one wave per
// workgroup polls the partition table's epoch exactly like a tenant
// workgroup polls its owner word (system scope: pinned host table; agent
// scope: device copy) and acknowledges every new epoch it sees into its own
// word of a pinned host array.  The host times "decision -> every workgroup
// observed it".  Every wave leaves at the stop epoch or after max_ticks of
// the 100 MHz wall clock, so the grid always drains.
__global__ __launch_bounds__(64) void k_switch_probe(const PartTable* t, u32 devtable, u32* acks, u32 stop,
                                                     u64 max_ticks) {
  if (threadIdx.x != 0) return;
  const u64 t0 = wall_clock64();
  u32 last = 0xFFFFFFFEu;
  for (;;) {
    const u32 e = devtable ? __hip_atomic_load(&t->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : __hip_atomic_load(&t->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (e != last) {
      last = e;
      __hip_atomic_store(&acks[blockIdx.x], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (e == stop || wall_clock64() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(1);
  }
}

int gpbs_hip_switch_probe(const void* table, int devtable, unsigned* acks, int nwg, unsigned stop,
                          unsigned long long max_ticks, hipStream_t s) {
  if (nwg <= 0 || nwg > 65536) return -22;
  hipLaunchKernelGGL(k_switch_probe, dim3(nwg), dim3(64), 0, s, (const PartTable*)table, (u32)devtable, acks, stop,
                     (u64)max_ticks);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_partition_switch(void* table, unsigned epoch, const unsigned* owners, hipStream_t s) {
  Owners ow;
  for (int i = 0; i < kXcds * kCtx; ++i) ow.o[i] = owners[i];
  hipLaunchKernelGGL(k_partition_switch, dim3(1), dim3(64), 0, s, (PartTable*)table, epoch, ow);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_counter_reduce(void* cnt, void* prev, const int* ids, int n, void* out, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_counter_reduce, dim3(n), dim3(64), 0, s, (u64*)cnt, (u64*)prev, ids, n, (u64*)out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_adapt(void* states, const void* deltas, const void* spin_sum, const void* spin_cnt, int n,
                   const gpbs_adapt_params_t* p, int* dirs, hipStream_t s) {
  if (n <= 0) return 0;
  DevParams dp;
  static_assert(sizeof(dp) == sizeof(gpbs_adapt_params_t), "params layout");
  __builtin_memcpy(&dp, p, sizeof(dp));
  hipLaunchKernelGGL(k_adapt, dim3((n + 63) / 64), dim3(64), 0, s, (gpbs_adapt_state_t*)states, (const u64*)deltas,
                     (const u64*)spin_sum, (const u64*)spin_cnt, n, dp, dirs);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // extern "C"
