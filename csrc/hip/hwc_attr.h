// Ownership attribution of live hardware counters to tenants (the per-vCPU
// PMU save/restore of X:xen/arch/x86/pmustate.c:87-111 done in space): the
// input is one sampler snapshot -- cumulative per-(XCD, SE) and per-XCD
// counters plus the cumulative ns every tenant owned every partition -- and
// the state the previous snapshot left; the output is each tenant's
// attributed deltas (pro rata to owned time) and the part of them that came
// from settled exclusive-ownership windows (what the PBS metric sees).
//
// Two implementations of one algorithm: hwc_attr_host (C++, the reference
// and the fallback) and k_hwc_attribute (csrc/hip/sched_kernels.hip, one
// workgroup, a thread per tenant / partition), which runs on the GPU on the
// headline path (csrc/hip/runtime.cpp, hwc_tenant_deltas).  Both sum in the
// same order; tests/test_gpu_kernels.py compares them on random inputs.
#pragma once
#include <cstddef>
#include <cstdint>

#include "common.hpp"

namespace gpbs_hip {

constexpr int kAttrP = kXcds * kCtx;  // partitions: (XCD, shader engine)

struct HwcAttrIn {
  u64 se_cur[kAttrP * kNumPmc];          // cumulative, SE-resolved slots
  u64 x_cur[kXcds * kNumPmc];            // cumulative, per XCD (every slot)
  long long own_cur[kMaxTenants * kAttrP];  // cumulative owned ns, [tenant][partition]
  u32 slot_se[kNumPmc];                  // slot k resolved per shader engine
  u32 se_mode;                           // partitions are exclusive shader engines
  u32 clean_pct;                         // exclusive-ownership window threshold (%), 0: pro rata
  u32 shared;                            // class-share time in the interval (no clean windows)
  u32 prime;                             // 1: only record the snapshot as the new previous one
  u32 nt_hi;                             // rows t >= nt_hi of own_cur are zero (and were: owned time only grows);
                                         // the device path reads rows < nt_hi only (0 = all rows)
  u32 drained;                           // bit p: partition p's last owner change was at least the drain
                                         // guard before this interval began (its previous owner is gone)
};

// The prefix of a snapshot the device path reads (rows < nt_hi of own_cur).
inline size_t hwc_attr_in_bytes(const HwcAttrIn& in) {
  const u32 rows = (in.nt_hi == 0 || in.nt_hi > (u32)kMaxTenants) ? (u32)kMaxTenants : in.nt_hi;
  return offsetof(HwcAttrIn, own_cur) + (size_t)rows * kAttrP * sizeof(long long);
}

struct HwcAttrPrev {  // carried from one snapshot to the next
  u64 se[kAttrP * kNumPmc];
  u64 x[kXcds * kNumPmc];
  long long own[kMaxTenants * kAttrP];
  int prev_raw[kAttrP];  // per partition: its >= clean_pct owner over the previous interval, -1 none
  int pad[kAttrP];
};

struct HwcAttrOut {
  double add[kMaxTenants][kNumPmc];   // attributed (pro rata to owned time)
  double addc[kMaxTenants][kNumPmc];  // of which from settled exclusive windows
  double hw_sum[kNumPmc];             // all hardware counts of the interval
  double unatt[kNumPmc];              // counts no owner explains
  u32 valid;                          // 0: a priming call (no deltas)
  u32 pad[3];                         // device path: [0] / [1] = 100 MHz wall clock at kernel entry / exit
};

__host__ __device__ inline u64 attr_dpos(u64 a, u64 b) { return a >= b ? a - b : 0; }  // Q5

// HwcAttrIn::drained for the interval (used_t, snap_t] (host): bit p when the
// partition's owner at the interval's first sample had held it for at least
// `guard` (its predecessor's tiles are gone) AND that owner is the only one
// that can be the interval's >= clean_pct owner -- no owner change landed in
// the first (100 - clean_pct) % of the interval.  A change there hands the
// window to a new owner whose predecessor was still running and draining at
// its head (with only the first condition, up to 20 % of another
// tenant's counts reached the new owner's clean window).  used_chg / snap_chg:
// each partition's last owner-change time as of the opening / closing sample.
// Intervals shorter than three guards get no bits: a drain that outlasts the
// guard must stay a small part of the window.
inline u32 hwc_drained_bits(int64_t used_t, int64_t snap_t, const int64_t* used_chg, const int64_t* snap_chg,
                            int64_t guard, u32 clean_pct) {
  if (used_t <= 0 || snap_t - used_t < 3 * guard) return 0;
  const int64_t span = snap_t - used_t;
  const int64_t head = clean_pct <= 100 ? (int64_t)(100 - clean_pct) : 0;
  u32 dr = 0;
  for (int p = 0; p < kAttrP; ++p) {
    if (used_t - used_chg[p] < guard) continue;
    const int64_t chg = snap_chg[p];
    if (chg > used_t && (chg - used_t) * 100 <= head * span) continue;
    dr |= 1u << p;
  }
  return dr;
}

inline void hwc_attr_prev_init(HwcAttrPrev& st) {
  for (int i = 0; i < kAttrP * kNumPmc; ++i) st.se[i] = 0;
  for (int i = 0; i < kXcds * kNumPmc; ++i) st.x[i] = 0;
  for (int i = 0; i < kMaxTenants * kAttrP; ++i) st.own[i] = 0;
  for (int i = 0; i < kAttrP; ++i) st.prev_raw[i] = -1;
}

inline void hwc_attr_record(const HwcAttrIn& in, HwcAttrPrev& st) {
  for (int i = 0; i < kAttrP * kNumPmc; ++i) st.se[i] = in.se_cur[i];
  for (int i = 0; i < kXcds * kNumPmc; ++i) st.x[i] = in.x_cur[i];
  for (int i = 0; i < kMaxTenants * kAttrP; ++i) st.own[i] = in.own_cur[i];
}

// Host reference.
//  * SE-resolved slots in SE-exclusive mode: partition (x, e)'s delta goes to
//    the tenants that owned it in the interval, pro rata to owned time.
//  * Other slots / co-resident modes: an XCD's delta is split by owned time
//    over its contexts; LLC misses (TCC, per XCD) by each tenant's attributed
//    share of the XCD's L2 requests.
//  * Clean (metric) part: a partition counts only when one tenant owned it
//    for >= clean_pct % of this interval AND its previous owner had drained
//    before the interval began -- either the same tenant held it over the
//    previous interval too, or its last owner change was at least the drain
//    guard before this interval's first sample (bit p of `drained`: the
//    switch-aligned sampler takes that sample right after the guard, so the
//    window of a new owner's tenure opens clean); a revoked tenant's draining
//    workgroups never land in the next owner's window.  XCD-wide counts are
//    clean only with one owner on the XCD.
inline void hwc_attr_host(const HwcAttrIn& in, HwcAttrPrev& st, HwcAttrOut& out) {
  constexpr int P = kAttrP, T = kMaxTenants;
  for (int t = 0; t < T; ++t)
    for (int k = 0; k < kNumPmc; ++k) out.add[t][k] = out.addc[t][k] = 0.0;
  for (int k = 0; k < kNumPmc; ++k) out.hw_sum[k] = out.unatt[k] = 0.0;
  out.valid = 0;
  if (in.prime) {
    hwc_attr_record(in, st);
    return;
  }
  static thread_local double own_d[T * P];
  for (int i = 0; i < T * P; ++i) {
    const long long d = in.own_cur[i] - st.own[i];
    own_d[i] = d > 0 ? (double)d : 0.0;
  }
  double tot_p[P];
  double span = 0;
  for (int p = 0; p < P; ++p) {
    double tot = 0;
    for (int t = 0; t < T; ++t) tot += own_d[t * P + p];
    tot_p[p] = tot;
    span = span > tot ? span : tot;
  }
  int clean_owner[P];
  for (int p = 0; p < P; ++p) {
    int raw = -1;
    if (span > 0 && !in.shared)
      for (int t = 0; t < T; ++t)
        if (own_d[t * P + p] * 100.0 >= span * in.clean_pct) raw = t;
    clean_owner[p] = (raw >= 0 && (((in.drained >> p) & 1u) || st.prev_raw[p] == raw)) ? raw : -1;
    st.prev_raw[p] = raw;
  }
  int xcd_owner[kXcds];
  for (int x = 0; x < kXcds; ++x) {
    int o = -1;
    bool ok = true;
    for (int e = 0; e < kCtx && ok; ++e) {
      const int p = x * kCtx + e;
      if (tot_p[p] <= 0) continue;
      ok = clean_owner[p] >= 0 && (o < 0 || o == clean_owner[p]);
      o = clean_owner[p];
    }
    xcd_owner[x] = ok ? o : -1;
  }
  static thread_local double refs_x[T][kXcds], refs_cx[T][kXcds];
  for (int t = 0; t < T; ++t)
    for (int x = 0; x < kXcds; ++x) refs_x[t][x] = refs_cx[t][x] = 0.0;
  for (int k = 0; k < kNumPmc; ++k) {
    const bool miss_by_refs = k == 3;
    if (in.se_mode && in.slot_se[k]) {
      for (int x = 0; x < kXcds; ++x)
        for (int e = 0; e < kCtx; ++e) {
          const int p = x * kCtx + e;
          const double v = (double)attr_dpos(in.se_cur[p * kNumPmc + k], st.se[p * kNumPmc + k]);
          out.hw_sum[k] += v;
          const double tot = tot_p[p];
          if (tot <= 0) {
            out.unatt[k] += v;
            continue;
          }
          for (int t = 0; t < T; ++t) {
            const double w = own_d[t * P + p];
            if (w <= 0) continue;
            const double a = v * w / tot;
            out.add[t][k] += a;
            if (k == 2) refs_x[t][x] += a;
            if (clean_owner[p] == t) {
              out.addc[t][k] += a;
              if (k == 2) refs_cx[t][x] += a;
            }
          }
        }
      continue;
    }
    for (int x = 0; x < kXcds; ++x) {
      const double v = (double)attr_dpos(in.x_cur[x * kNumPmc + k], st.x[x * kNumPmc + k]);
      out.hw_sum[k] += v;
      double wt[T], tot = 0;
      bool by_refs = false;
      if (miss_by_refs) {
        for (int t = 0; t < T; ++t) tot += (wt[t] = refs_x[t][x]);
        by_refs = tot > 0;
      }
      if (!by_refs) {  // time share over every context of the XCD
        tot = 0;
        for (int t = 0; t < T; ++t) {
          double s = 0;
          for (int e = 0; e < kCtx; ++e) s += own_d[t * P + x * kCtx + e];
          wt[t] = s;
          tot += s;
        }
      }
      if (tot <= 0) {
        out.unatt[k] += v;
        continue;
      }
      for (int t = 0; t < T; ++t)
        if (wt[t] > 0) {
          const double a = v * wt[t] / tot;
          out.add[t][k] += a;
          if (k == 2) refs_x[t][x] += a;
          if (miss_by_refs && in.se_mode && in.slot_se[2])
            out.addc[t][k] += v * refs_cx[t][x] / tot;
          else if (xcd_owner[x] == t)
            out.addc[t][k] += a;
        }
    }
  }
  hwc_attr_record(in, st);
  out.valid = 1;
}

}  // namespace gpbs_hip
