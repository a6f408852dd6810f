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
//                        to tenants (csrc/hip/hwc_attr.h): one workgroup,
//                        the snapshot staged into LDS in one pass of wide
//                        loads, 8-lane reductions / ballots per partition, a
//                        lane per tenant and a wave per counter slot; the
//                        previous snapshot stays resident in device memory.
#include <cstddef>

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
    const u64 c = __hip_atomic_load(cnt + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
      scale, strict_ref, grow_pct;
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


// One workgroup of 256 threads (4 waves); lane = tenant (kMaxTenants == the
// 64-lane wavefront).  The host copies the live rows of the snapshot to
// device memory first (hipMemcpyAsync; round 3 read pinned host memory inside
// the per-tenant loops: 78 us per call); the kernel stages them into LDS with
// every 16-byte load in flight at once.  Then
//   * per-partition owned-time totals: 8 threads per partition, a 3-step
//     butterfly (integer ns: exact in any order);
//   * clean owners: the last tenant over the clean_pct threshold, from a
//     wave ballot per partition;
//   * everything lane-independent once: per-XCD owners and totals, each
//     (partition, SE slot)'s count times its partition's reciprocal, the
//     per-slot hardware sums, slot 2's attributable L2 requests per XCD;
//   * attribution: wave k attributes counter slot k for all 64 tenants at
//     once, the four waves independently (wave 3 splits the L2 misses by its
//     lane's slot-2 shares, a few FMAs per XCD in registers).
// The previous snapshot and the clean-owner history stay in device memory.
struct AttrArgs {  // the snapshot's scalars, by value (no dependent load before the staging loads)
  u32 slot_se[kNumPmc];
  u32 se_mode, clean_pct, shared, prime, nt_hi, drained;
};

__global__ __launch_bounds__(256) void k_hwc_attribute(const HwcAttrIn* __restrict__ in, HwcAttrPrev* __restrict__ st,
                                                       HwcAttrOut* __restrict__ out, AttrArgs args) {
  __builtin_amdgcn_s_setprio(3);
  const u32 t_entry = (u32)__builtin_amdgcn_s_memrealtime();  // 100 MHz: the kernel's own duration -> out->pad
  constexpr int P = kAttrP, T = kMaxTenants, X = kXcds, K = kNumPmc, E = kCtx;
  static_assert(T == 64 && X * E == P && P * T == 8 * 256, "one wave of tenants, 8 owned-time words per thread");
  static_assert(offsetof(HwcAttrIn, x_cur) == offsetof(HwcAttrIn, se_cur) + sizeof(u64) * P * K &&
                    offsetof(HwcAttrPrev, x) == offsetof(HwcAttrPrev, se) + sizeof(u64) * P * K,
                "se and x counters adjacent: one 160-word array");
  static_assert(offsetof(HwcAttrIn, own_cur) % 16 == 0 && offsetof(HwcAttrPrev, own) % 16 == 0, "16-byte loads");
  constexpr int NC = (P + X) * K / 2;  // 16-byte counter loads (80)
  __shared__ double ownT[P][T + 1];    // owned ns of the interval, [partition][tenant], padded
  __shared__ double vse[P][K], vx[X][K];
  __shared__ double tot_p[P], inv_p[P], tot_x[X], inv_x[X], vsc[P][K], refx[X], inv_refx[X];
  __shared__ int clean_owner[P], xcd_owner[X];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const u32 prime = args.prime;
  // 1. stage: every load of the snapshot and of the previous state in flight at once
  const longlong2* oc = reinterpret_cast<const longlong2*>(in->own_cur);
  longlong2* op = reinterpret_cast<longlong2*>(st->own);
  const ulonglong2* cc = reinterpret_cast<const ulonglong2*>(in->se_cur);
  ulonglong2* cp = reinterpret_cast<ulonglong2*>(st->se);
  longlong2 c[4], q[4];
  ulonglong2 cv{}, qv{};
  // only the rows of tenants that ever owned a partition (copied by the host)
  const u32 nth = args.nt_hi;
  const int nload = (nth == 0 || nth > (u32)T) ? T * P / 2 : (int)nth * P / 2;  // 16-byte loads
#pragma unroll
  for (int j = 0; j < 4; ++j) c[j] = j * 256 + tid < nload ? oc[j * 256 + tid] : longlong2{0, 0};
  if (tid < NC) cv = cc[tid];
  const u32 se_mode = args.se_mode, clean_pct = args.clean_pct, shared = args.shared;
  u32 slot_se[K];
#pragma unroll
  for (int k = 0; k < K; ++k) slot_se[k] = args.slot_se[k];
  if (!prime) {
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j] = j * 256 + tid < nload ? op[j * 256 + tid] : longlong2{0, 0};
    if (tid < NC) qv = cp[tid];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = (j * 256 + tid) * 2, t = i / P, p = i % P;
      const long long d0 = c[j].x - q[j].x, d1 = c[j].y - q[j].y;
      ownT[p][t] = d0 > 0 ? (double)d0 : 0.0;
      ownT[p + 1][t] = d1 > 0 ? (double)d1 : 0.0;
    }
    if (tid < NC) {
      const int i = tid * 2;
      double* dst = i < P * K ? &vse[0][0] + i : &vx[0][0] + (i - P * K);
      dst[0] = (double)attr_dpos(cv.x, qv.x);
      dst[1] = (double)attr_dpos(cv.y, qv.y);
    }
  }
  // the new previous snapshot (each thread overwrites only what it read)
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j * 256 + tid < nload) op[j * 256 + tid] = c[j];
  if (tid < NC) cp[tid] = cv;
  if (prime) {
    if (tid == 0) out->valid = 0u;
    return;
  }
  __syncthreads();
  // 2. owned-time totals per partition: 8 threads per partition sum 8
  // tenants each, then a 3-step butterfly (the owned ns are integers, so the
  // totals are exact in any order) -- 3 cross-lane steps instead of a 6-step
  // wave reduction per partition, and the 32 reciprocals in parallel
  {
    static_assert(P * 8 == 256 && T == 64, "8 threads x 8 tenants per partition");
    const int p = tid >> 3, part = tid & 7;
    double s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += ownT[p][part * 8 + j];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if (part == 0) {
      tot_p[p] = s;
      inv_p[p] = s > 0 ? 1.0 / s : 0.0;
    }
  }
  __syncthreads();
  // 3. clean owners: >= clean_pct of the interval's span, and the previous
  // owner drained before the interval (the same owner as the previous
  // interval, or the last owner change a drain guard before it: args.drained)
  double span = 0;
#pragma unroll
  for (int p = 0; p < P; ++p) span = span > tot_p[p] ? span : tot_p[p];
#pragma unroll
  for (int i = 0; i < P / 4; ++i) {
    const int p = wave * (P / 4) + i;
    const bool over = span > 0 && !shared && ownT[p][lane] * 100.0 >= span * clean_pct;
    const unsigned long long m = __ballot(over);
    if (lane == 0) {
      const int raw = m ? 63 - __builtin_clzll(m) : -1;  // the host keeps the last tenant over the bar
      clean_owner[p] = (raw >= 0 && (((args.drained >> p) & 1u) || st->prev_raw[p] == raw)) ? raw : -1;
      st->prev_raw[p] = raw;
    }
  }
  __syncthreads();
  // 3b. everything lane-independent, once: per-XCD owners and totals (threads
  // 0-7), each (partition, SE slot)'s count scaled by its partition's
  // reciprocal (64-191), the per-slot hardware sums / unexplained counts
  // (192-195) and slot 2's attributable L2 requests per XCD (200-207, the
  // denominator of the miss split -- the sum over tenants of their slot-2
  // shares, so no wave reduction is needed for it)
  const bool se2 = se_mode && slot_se[2];
  auto refs_tot = [&](const int x) {
    double r = 0;
    if (se2) {
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (tot_p[x * E + e] > 0) r += vse[x * E + e][2];
    } else {
      double tx = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) tx += tot_p[x * E + e];
      if (tx > 0) r = vx[x][2];
    }
    return r;
  };
  if (tid < X) {
    int o = -1;
    bool ok = true;
    for (int e = 0; e < E && ok; ++e) {
      const int p = tid * E + e;
      if (tot_p[p] <= 0) continue;
      ok = clean_owner[p] >= 0 && (o < 0 || o == clean_owner[p]);
      o = clean_owner[p];
    }
    xcd_owner[tid] = ok ? o : -1;
    // an XCD's owned time over its shader engines (exact: integer ns)
    double tx = 0;
    for (int e = 0; e < E; ++e) tx += tot_p[tid * E + e];
    tot_x[tid] = tx;
    inv_x[tid] = tx > 0 ? 1.0 / tx : 0.0;
  } else if (tid >= 64 && tid < 64 + P * K) {
    const int p = (tid - 64) / K, k = (tid - 64) % K;
    vsc[p][k] = tot_p[p] > 0 ? vse[p][k] * inv_p[p] : 0.0;
  } else if (tid >= 192 && tid < 192 + K) {
    const int k = tid - 192;
    double hs = 0, ua = 0;
    if (se_mode && slot_se[k]) {
      for (int p = 0; p < P; ++p) {
        hs += vse[p][k];
        if (tot_p[p] <= 0) ua += vse[p][k];
      }
    } else {
      for (int x = 0; x < X; ++x) {
        double tx = 0;
        for (int e = 0; e < E; ++e) tx += tot_p[x * E + e];
        const double tot = (k == 3 && refs_tot(x) > 0) ? 1.0 : tx;
        hs += vx[x][k];
        if (tot <= 0) ua += vx[x][k];
      }
    }
    out->hw_sum[k] = hs;
    out->unatt[k] = ua;
  } else if (tid >= 200 && tid < 200 + X) {
    const double r = refs_tot(tid - 200);
    refx[tid - 200] = r;
    inv_refx[tid - 200] = r > 0 ? 1.0 / r : 0.0;
  }
  __syncthreads();
  // 4. attribution, lane = tenant, wave k = counter slot k; the four waves
  // never wait for each other: wave 3's L2 misses are split by this lane's
  // slot-2 shares, which it recomputes in registers (a few FMAs per XCD)
  const int t = lane;
  const int k = wave;
  double add = 0, addc = 0;
  if (se_mode && slot_se[k]) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const double a = ownT[p][t] * vsc[p][k];  // 0 for an unowned partition or an idle tenant
      add += a;
      if (clean_owner[p] == t) addc += a;
    }
  } else {
    const bool miss_by_refs = k == 3;
#pragma unroll
    for (int x = 0; x < X; ++x) {
      const double v = vx[x][k];
      double wt = 0, inv = inv_x[x], rcx = 0;
      bool by_refs = false;
      if (miss_by_refs && refx[x] > 0) {  // this lane's slot-2 share on XCD x
        by_refs = true;
        inv = inv_refx[x];
        if (se2) {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const int p = x * E + e;
            const double a = ownT[p][t] * vsc[p][2];
            wt += a;
            if (clean_owner[p] == t) rcx += a;
          }
        } else {
          double w = 0;
#pragma unroll
          for (int e = 0; e < E; ++e) w += ownT[x * E + e][t];
          wt = vx[x][2] * w * inv_x[x];
        }
      }
      if (!by_refs) {
        if (tot_x[x] <= 0) continue;
#pragma unroll
        for (int e = 0; e < E; ++e) wt += ownT[x * E + e][t];
      }
      if (wt <= 0) continue;
      const double a = v * wt * inv;
      add += a;
      if (miss_by_refs && se2)
        addc += v * rcx * inv;
      else if (xcd_owner[x] == t)
        addc += a;
    }
  }
  out->add[t][k] = add;
  out->addc[t][k] = addc;
  __syncthreads();
  if (tid == 0) {
    out->pad[0] = t_entry;
    out->pad[1] = (u32)__builtin_amdgcn_s_memrealtime();
    out->valid = 1u;
  }
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

// Ownership attribution of one counter snapshot.  h_in: the snapshot in
// pinned host memory; d_in: a device staging buffer (HwcAttrIn-sized) -- the
// counters and the live tenants' owned-time rows are copied there first
// (one DMA-sized copy on the same stream) so the kernel's loads never wait
// on PCIe; the scalars travel as kernel arguments.  st: device HwcAttrPrev;
// out: host-visible HwcAttrOut.
// copy 0: d_in already holds the snapshot (the runtime wrote it into
// fine-grained VRAM through the BAR), so no copy runs on the GPU
int gpbs_hip_hwc_attribute2(const void* h_in, void* d_in, void* st, void* out, hipStream_t s, int copy) {
  const HwcAttrIn* hin = (const HwcAttrIn*)h_in;
  AttrArgs a{};
  for (int k = 0; k < kNumPmc; ++k) a.slot_se[k] = hin->slot_se[k];
  a.se_mode = hin->se_mode;
  a.clean_pct = hin->clean_pct;
  a.shared = hin->shared;
  a.prime = hin->prime;
  a.nt_hi = hin->nt_hi;
  a.drained = hin->drained;
  if (copy && hipMemcpyAsync(d_in, h_in, hwc_attr_in_bytes(*hin), hipMemcpyHostToDevice, s) != hipSuccess) return -5;
  hipLaunchKernelGGL(k_hwc_attribute, dim3(1), dim3(256), 0, s, (const HwcAttrIn*)d_in, (HwcAttrPrev*)st,
                     (HwcAttrOut*)out, a);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_hwc_attribute(const void* h_in, void* d_in, void* st, void* out, hipStream_t s) {
  return gpbs_hip_hwc_attribute2(h_in, d_in, st, out, s, 1);
}

}  // extern "C"
