// PBS adaptive-quantum policy, host reference implementation.
// Behavior reference: X:xen/common/sched_credit.c:261-389 (built PBS) and
// X:xen/common/sched_credit_atc.c:210-460 (unbuilt ATC variant).
#include "adapt.h"

#include "adapt_impl.h"

#include <cstring>

namespace gpbs {

uint32_t adapt_dec(uint32_t t, const AdaptParams& p) { return impl::dec(t, p); }
uint32_t adapt_inc(uint32_t t, const AdaptParams& p) { return impl::inc(t, p); }

void adapt_init(AdaptState& s, const AdaptParams& p, uint32_t default_tslice_us) {
  std::memset(&s, 0, sizeof(s));
  s.tslice_us = default_tslice_us;                       // csched_dom_init :1217
  s.tick_period_us = default_tslice_us / p.ticks_per_tslice;
  s.window_left = kWindow;
  s.phase = kPhaseLow;
}

int adapt_update(AdaptState& s, const AdaptParams& p, uint64_t inst, uint64_t miss, uint64_t spin_sum,
                 uint64_t spin_count, bool* rearm) {
  const int r = impl::update(s, p, inst, miss, spin_sum, spin_count);
  if (rearm) *rearm = (r & 4) != 0;
  return (r & 3) - 1;
}

// ------------------------------------------------------------------ ATC ----

uint32_t atc_bucket(uint64_t x) {
  static const uint64_t edges[10] = {1024, 1536, 2048, 3072, 4096, 6144, 8192, 12288, 16384, 32768};
  if (x < 1024) return 1;
  uint32_t i = 0;
  for (; i < 10; ++i)
    if (x < edges[i]) break;
  return i + 6;
}

void atc_init(AtcState& s, const AtcParams& p) {
  std::memset(&s, 0, sizeof(s));
  s.tslice_us = p.default_us;  // csched_dom_init (atc) :1409-1417
  s.count = p.warmup;
  s.hist[0].tslice = s.tslice_us;
}

void atc_report(AtcState& s, const AtcParams& p, uint64_t wait) {
  if (p.wait_unit_ns > 1) wait /= p.wait_unit_ns;
  s.spin = s.spin / p.alpha + wait / p.alpha * (p.alpha - 1);
  s.spin_count++;
}

namespace {
inline void shift(AtcState& s) {
  s.hist[0] = s.hist[1];
  s.hist[1] = s.hist[2];
  s.hist[2] = s.hist[3];
}
inline uint32_t climb_down(uint32_t prev, const AtcParams& p) {
  return prev >= p.climb_floor_us ? prev - p.climb_step_us : p.min_us;
}
}  // namespace

void atc_update(AtcState& s, const AtcParams& p) {
  const uint32_t b = atc_bucket(s.spin);
  if (s.spin_count <= 1 && b == 1) {
    // Quiet tenant: lengthen the slice (:300-330).
    s.zero_count++;
    s.prev_spin_count = s.spin_count;
    s.spin_count = 0;
    s.spin = 0;
    s.tslice_us = s.tslice_us < p.max_us - p.zero_step_us ? s.tslice_us + p.zero_step_us : p.max_us;
    if (s.count == 0) {
      shift(s);
      // Q10 fix: the reference pushes an uninitialised local; push the slice.
      s.hist[3].bucket = b;
      s.hist[3].tslice = s.tslice_us;
    }
    return;
  }
  uint32_t t;
  if (s.count > 0) {
    if (b == 1)
      t = p.max_us;
    else if (b <= 15)
      t = p.base_us - p.slope_us * b;
    else
      t = p.min_us;
    s.hist[p.warmup - s.count].bucket = b;
    s.hist[p.warmup - s.count].tslice = t;
    s.count--;
  } else if (s.hist[2].bucket < b) {
    shift(s);
    s.hist[3].bucket = b;
    s.hist[3].tslice = climb_down(s.hist[2].tslice, p);
    t = s.hist[3].tslice;
  } else if (s.hist[2].bucket == b) {
    shift(s);
    s.hist[3].bucket = b;
    s.hist[3].tslice = s.hist[2].tslice;
    t = s.hist[3].tslice;
  } else {
    const bool falling = s.hist[0].bucket >= s.hist[1].bucket && s.hist[1].tslice >= s.hist[2].tslice;
    shift(s);
    s.hist[3].bucket = b;
    s.hist[3].tslice = falling ? climb_down(s.hist[2].tslice, p) : s.hist[2].tslice;
    t = s.hist[3].tslice;
  }
  s.prev_spin_count = s.spin_count;
  s.spin_count = 0;
  s.tslice_us = t;
}

}  // namespace gpbs
