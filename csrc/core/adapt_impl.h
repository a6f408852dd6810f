// Single-source PBS adaptation step, compiled both by g++ (host engine,
// csrc/core/adapt.cpp) and by hipcc for gfx950 (batched device kernel,
// csrc/hip/sched_kernels.hip).  Integer-only; C truncating division.
// Reference: X:xen/common/sched_credit.c:286-389.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define GPBS_HD __attribute__((host, device)) inline
#else
#define GPBS_HD inline
#endif

namespace gpbs {
namespace impl {

template <class P>
GPBS_HD uint64_t trunc_spin(uint64_t v, const P& p) { return p.strict_ref ? (uint16_t)v : v; }
template <class P>
GPBS_HD uint64_t trunc_u32(uint64_t v, const P& p) { return p.strict_ref ? (uint32_t)v : v; }
template <class P>
GPBS_HD int64_t rate_int(uint64_t v, const P& p) { return p.strict_ref ? (int64_t)(int32_t)v : (int64_t)v; }

template <class P>
GPBS_HD uint32_t dec(uint32_t t, const P& p) {
  if (t >= p.switch_boundary * 3) return t / (3 * p.inc_us) * p.inc_us;  // /3 in quantum units (reference: /300*100)
  return t >= p.min_us + p.dec_us ? t - p.dec_us : p.min_us;
}

// grow_pct > 0 (MI355X profile): proportional growth, at least inc_us -- a
// 1 -> 11 ms climb in 4 stable steps instead of 10, because on time-shared
// GPU partitions a tenant's metric updates arrive once per clean counter
// window (5-10 ms), not every 1 ms tick, and a phase lasts a few hundred ms.
// (Growing while the window refills too was tried: it put the gang-switched
// memory region out of step for good -- tests/test_se_mode.py, 0.5 aligned.)
template <class P>
GPBS_HD uint32_t inc(uint32_t t, const P& p) {
  uint32_t n = t + p.inc_us;
  if (p.grow_pct) {
    const uint64_t m = (uint64_t)t * (100 + p.grow_pct) / 100;
    if (m > n) n = m > p.max_us ? p.max_us : (uint32_t)m;
  }
  return n >= p.max_us ? p.max_us : n;
}

template <class E, class P>
GPBS_HD void put(E& e, const P& p, uint64_t spin, uint64_t inst, uint64_t miss) {
  e.spin = trunc_spin(spin, p);
  e.inst = trunc_u32(inst, p);
  e.miss = trunc_u32(miss, p);
}

// S: AdaptState-like {tslice_us, tick_period_us, window_left, stable_count,
// phase, last_err, last_curr, last_win, filter[5]{spin,inst,miss}}.
// Returns (dir + 1) | (rearm ? 4 : 0) where dir is +1/-1/0 (quantum grew/shrank/kept).
template <class S, class P>
GPBS_HD int update(S& s, const P& p, uint64_t inst, uint64_t miss, uint64_t spin_sum, uint64_t spin_count) {
  constexpr int W = 5;
  const uint32_t before = s.tslice_us;
  int rearm = 0;
  const int64_t thr = p.threshold;
  const int64_t curr = inst ? rate_int(miss * p.scale / inst, p) : 0;
  const uint64_t avg_spin = spin_count ? spin_sum / spin_count : 0;
  s.last_curr = curr;
  if (s.window_left > 0) {
    put(s.filter[W - s.window_left], p, avg_spin, inst, miss);
    s.window_left--;
    if (curr > 0 && curr < thr) s.tslice_us = dec(s.tslice_us, p);
    s.last_win = -1;
    s.last_err = -1;
  } else {
    uint64_t isum = 0, msum = 0;
    for (int i = 0; i < W; ++i) {
      isum += s.filter[i].inst;
      msum += s.filter[i].miss;
    }
    const uint64_t inst_mean = isum / W;
    const uint64_t miss_mean = msum / W;
    const int64_t win = inst_mean ? rate_int(miss_mean * p.scale / inst_mean, p) : 0;
    int64_t err;
    if (win > 0)
      err = p.strict_ref ? (int64_t)(int32_t)(curr * 100 / win) : curr * 100 / win;
    else
      err = curr == 0 ? 100 : 0;
    s.last_win = win;
    s.last_err = (int32_t)err;
    const bool stable = (err >= (int64_t)p.band_lo && err <= (int64_t)p.band_hi) ||
                        (err > (int64_t)p.band_hi && win >= thr) || (curr < thr && win < thr);
    if (stable) {
      s.stable_count++;
      for (int i = 0; i < W - 1; ++i) s.filter[i] = s.filter[i + 1];
      put(s.filter[W - 1], p, avg_spin, inst, miss);
      if (win >= thr) {
        s.phase = 1;  // cache-sensitive: hold the partition longer
        s.tslice_us = inc(s.tslice_us, p);
      } else {
        s.phase = 2;
        s.tslice_us = dec(s.tslice_us, p);
      }
      s.tick_period_us = s.tslice_us / p.ticks_per_tslice;  // Q9: stable branch only
    } else {
      s.stable_count = 0;
      for (int i = 0; i < W; ++i) s.filter[i].spin = s.filter[i].inst = s.filter[i].miss = 0;
      put(s.filter[0], p, avg_spin, inst, miss);
      s.window_left = W - 1;
      if (curr < thr) s.tslice_us = dec(s.tslice_us, p);
      rearm = 4;
    }
  }
  const int dir = s.tslice_us > before ? 1 : (s.tslice_us < before ? -1 : 0);
  return (dir + 1) | rearm;
}

}  // namespace impl
}  // namespace gpbs
