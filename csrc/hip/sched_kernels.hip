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
//   k_hwc_attribute    : ownership attribution of one live-counter snapshot
//                        to tenants (csrc/hip/hwc_attr.h): one workgroup, a
//                        thread per partition for the ownership reductions
//                        and a thread per tenant for the attribution; the
//                        previous snapshot stays resident in device memory.
#include "common.hpp"
#include "hwc_attr.h"
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


// One workgroup of 256 threads (4 waves).  Threads p < 32 reduce ownership
// per partition, threads t < 64 attribute per tenant; every sum runs in the
// order of hwc_attr_host.  The input is the sampler's snapshot in pinned
// host memory (read once, ~17 KB); the previous snapshot and the per-
// partition clean-owner history live in device memory between launches.
__global__ __launch_bounds__(256) void k_hwc_attribute(const HwcAttrIn* __restrict__ in, HwcAttrPrev* __restrict__ st,
                                                       HwcAttrOut* __restrict__ out) {
  __builtin_amdgcn_s_setprio(3);
  constexpr int P = kAttrP, T = kMaxTenants;
  __shared__ double own_d[T * P];  // 16 KiB
  __shared__ double tot_p[P];
  __shared__ double refs_x[T][kXcds], refs_cx[T][kXcds];
  __shared__ int clean_owner[P], xcd_owner[kXcds];
  __shared__ double span_s;
  __shared__ double hw_sum[kNumPmc], unatt[kNumPmc];
  const int tid = threadIdx.x;
  const u32 prime = in->prime;
  if (!prime) {
    for (int i = tid; i < T * P; i += 256) {
      const long long d = in->own_cur[i] - st->own[i];
      own_d[i] = d > 0 ? (double)d : 0.0;
    }
    for (int i = tid; i < T * kXcds; i += 256) {
      (&refs_x[0][0])[i] = 0.0;
      (&refs_cx[0][0])[i] = 0.0;
    }
    if (tid < kNumPmc) hw_sum[tid] = unatt[tid] = 0.0;
  }
  __syncthreads();
  if (!prime) {
    if (tid < P) {
      double tot = 0;
      for (int t = 0; t < T; ++t) tot += own_d[t * P + tid];
      tot_p[tid] = tot;
    }
    __syncthreads();
    if (tid == 0) {
      double span = 0;
      for (int p = 0; p < P; ++p) span = span > tot_p[p] ? span : tot_p[p];
      span_s = span;
    }
    __syncthreads();
    if (tid < P) {
      const double span = span_s;
      int raw = -1;
      if (span > 0 && !in->shared)
        for (int t = 0; t < T; ++t)
          if (own_d[t * P + tid] * 100.0 >= span * in->clean_pct) raw = t;
      clean_owner[tid] = (raw >= 0 && st->prev_raw[tid] == raw) ? raw : -1;
      st->prev_raw[tid] = raw;
    }
    __syncthreads();
    if (tid < kXcds) {
      int o = -1;
      bool ok = true;
      for (int e = 0; e < kCtx && ok; ++e) {
        const int p = tid * kCtx + e;
        if (tot_p[p] <= 0) continue;
        ok = clean_owner[p] >= 0 && (o < 0 || o == clean_owner[p]);
        o = clean_owner[p];
      }
      xcd_owner[tid] = ok ? o : -1;
    }
    __syncthreads();
    const u32 se_mode = in->se_mode;
    double add[kNumPmc] = {0, 0, 0, 0}, addc[kNumPmc] = {0, 0, 0, 0};
    for (int k = 0; k < kNumPmc; ++k) {
      const bool miss_by_refs = k == 3;
      if (se_mode && in->slot_se[k]) {
        if (tid == 0)  // interval totals (order of the host loop)
          for (int p = 0; p < P; ++p) {
            const double v = (double)attr_dpos(in->se_cur[p * kNumPmc + k], st->se[p * kNumPmc + k]);
            hw_sum[k] += v;
            if (tot_p[p] <= 0) unatt[k] += v;
          }
        if (tid < T) {
          const int t = tid;
          for (int x = 0; x < kXcds; ++x)
            for (int e = 0; e < kCtx; ++e) {
              const int p = x * kCtx + e;
              const double tot = tot_p[p];
              const double w = own_d[t * P + p];
              if (tot <= 0 || w <= 0) continue;
              const double v = (double)attr_dpos(in->se_cur[p * kNumPmc + k], st->se[p * kNumPmc + k]);
              const double a = v * w / tot;
              add[k] += a;
              if (k == 2) refs_x[t][x] += a;
              if (clean_owner[p] == t) {
                addc[k] += a;
                if (k == 2) refs_cx[t][x] += a;
              }
            }
        }
        __syncthreads();
        continue;
      }
      // per-XCD slot: weights need every tenant's row (written above, synced)
      if (tid < T) {
        const int t = tid;
        for (int x = 0; x < kXcds; ++x) {
          const double v = (double)attr_dpos(in->x_cur[x * kNumPmc + k], st->x[x * kNumPmc + k]);
          double tot = 0, wt = 0;
          bool by_refs = false;
          if (miss_by_refs) {
            for (int u = 0; u < T; ++u) tot += refs_x[u][x];
            by_refs = tot > 0;
            wt = refs_x[t][x];
          }
          if (!by_refs) {
            tot = 0;
            for (int u = 0; u < T; ++u) {
              double s = 0;
              for (int e = 0; e < kCtx; ++e) s += own_d[u * P + x * kCtx + e];
              tot += s;
              if (u == t) wt = s;
            }
          }
          if (t == 0) {
            hw_sum[k] += v;
            if (tot <= 0) unatt[k] += v;
          }
          if (tot <= 0 || wt <= 0) continue;
          const double a = v * wt / tot;
          add[k] += a;
          if (k == 2) refs_x[t][x] += a;  // own row only: read by others at k == 3, after the sync below
          if (miss_by_refs && se_mode && in->slot_se[2])
            addc[k] += v * refs_cx[t][x] / tot;
          else if (xcd_owner[x] == t)
            addc[k] += a;
        }
      }
      __syncthreads();
    }
    if (tid < T)
      for (int k = 0; k < kNumPmc; ++k) {
        out->add[tid][k] = add[k];
        out->addc[tid][k] = addc[k];
      }
    if (tid < kNumPmc) {
      out->hw_sum[tid] = hw_sum[tid];
      out->unatt[tid] = unatt[tid];
    }
  }
  __syncthreads();  // every read of the previous snapshot is done
  for (int i = tid; i < P * kNumPmc; i += 256) st->se[i] = in->se_cur[i];
  for (int i = tid; i < kXcds * kNumPmc; i += 256) st->x[i] = in->x_cur[i];
  for (int i = tid; i < T * P; i += 256) st->own[i] = in->own_cur[i];
  if (tid == 0) out->valid = prime ? 0u : 1u;
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

// Ownership attribution of one counter snapshot (in: host-visible HwcAttrIn;
// st: device HwcAttrPrev; out: host-visible HwcAttrOut).
int gpbs_hip_hwc_attribute(const void* in, void* st, void* out, hipStream_t s) {
  hipLaunchKernelGGL(k_hwc_attribute, dim3(1), dim3(256), 0, s, (const HwcAttrIn*)in, (HwcAttrPrev*)st,
                     (HwcAttrOut*)out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // extern "C"
