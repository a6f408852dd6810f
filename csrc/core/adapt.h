// PBS per-tenant phase detector and adaptive quantum (the policy delta of
// the reference, X:xen/common/sched_credit.c:261-389).
//
// Integer semantics (C truncating division) are reproduced exactly so that
// the host implementation, the batched HIP kernel (csrc/hip/adapt.hip) and the
// Python oracle (pbs_amd/core/oracle.py) agree bit for bit.  Constants that the
// reference hard-codes as #defines are runtime fields of AdaptParams whose
// defaults equal the reference.
#pragma once
#include <cstdint>

namespace gpbs {

constexpr int kWindow = 5;          // EVENT_TRACKING_WINDOW (sched_credit.c:114)
constexpr int kPhaseLow = 1;        // SPIN_LOW_PHASE  (cache-sensitive)
constexpr int kPhaseHigh = 2;       // SPIN_HIGH_PHASE (not cache-bound)

struct AdaptParams {
  uint32_t threshold = 100;      // misses per 100k instructions (1 MPKI), :345,355-360
  uint32_t band_lo = 70;         // err band, :354
  uint32_t band_hi = 130;
  uint32_t min_us = 100;         // :291
  uint32_t max_us = 1100;        // :299
  uint32_t inc_us = 100;         // :299
  uint32_t dec_us = 200;         // :291
  uint32_t switch_boundary = 900;  // SWITCH_BOUNDARY (x3 => divide-by-3 path), :112,288
  uint32_t ticks_per_tslice = 3;   // CSCHED_TICKS_PER_TSLICE, :46,372
  uint32_t spin_floor = 10000;     // spinlock mean filter, :333
  uint32_t scale = 100000;         // miss-rate scale (per 100k inst)
  // Reference truncates window entries to u16 spin / u32 inst / u32 miss
  // (struct event_sample, :176-181).  strict_ref=1 reproduces that (Q7);
  // strict_ref=0 keeps full 64-bit samples (GPU counter rates overflow u32).
  uint32_t strict_ref = 0;
  // gpbs extension (0 = the reference's additive steps): proportional growth
  // of the stable branch, grow_pct % per step (adapt_impl.h inc)
  uint32_t grow_pct = 0;
};

struct FilterEntry {
  uint64_t spin;
  uint64_t inst;
  uint64_t miss;
};

// Per-tenant adaptation state (subset of struct csched_dom, :196-220).
struct AdaptState {
  uint32_t tslice_us;
  uint32_t tick_period_us;
  uint32_t window_left;     // event_tracking_window
  uint32_t stable_count;    // event_stable_count
  uint32_t phase;
  int32_t last_err;         // diagnostics (trace ADAPT record)
  int64_t last_curr;
  int64_t last_win;
  FilterEntry filter[kWindow];
};

void adapt_init(AdaptState& s, const AdaptParams& p, uint32_t default_tslice_us = 100);
// One metric-tick update for one tenant. spin_sum/spin_count are the spin
// reports accumulated since the last tick (spinlock_metric_update/count).
// Returns +1 if the quantum grew, -1 if it shrank, 0 otherwise; *rearm set
// when the window was re-armed (phase change).
int adapt_update(AdaptState& s, const AdaptParams& p, uint64_t inst, uint64_t miss,
                 uint64_t spin_sum, uint64_t spin_count, bool* rearm);
uint32_t adapt_dec(uint32_t tslice, const AdaptParams& p);
uint32_t adapt_inc(uint32_t tslice, const AdaptParams& p);

// ---------------------------------------------------------------- ATC -----
// Spin-latency driven alternative policy (X:xen/common/sched_credit_atc.c).
struct AtcParams {
  uint32_t default_us = 30000;   // CSCHED_DEFAULT_TSLICE_US (atc :49)
  uint32_t min_us = 300;         // :313,362
  uint32_t max_us = 30000;
  uint32_t zero_step_us = 500;   // :307-313
  uint32_t climb_step_us = 1000; // :360-366
  uint32_t climb_floor_us = 1300;
  uint32_t base_us = 49980;      // :340-346 initial slice = base - slope*bucket
  uint32_t slope_us = 3300;
  uint32_t alpha = 4;            // EWMA alpha (:217)
  uint32_t warmup = 3;           // sdom->count (:1415)
  uint32_t apply_period_us = 21000;  // CSCHED_TIME_APPLY (:50)
  // Reported waits are ns (K10 probes time RCCL collectives and stream
  // syncs); the reference's buckets (:241-262) are in spin-loop iterations.
  // wait_unit_ns converts (0/1 = feed raw values, reference-exact).
  uint32_t wait_unit_ns = 0;
};

struct AtcHist {
  uint32_t bucket;
  uint32_t tslice;
};

struct AtcState {
  uint64_t spin;          // EWMA of reported wait
  uint64_t spin_count;
  uint64_t prev_spin_count;
  uint32_t count;         // warm-up samples left
  uint32_t zero_count;
  uint32_t tslice_us;
  uint32_t reserved;
  AtcHist hist[4];        // sstate[0..3]
};

uint32_t atc_bucket(uint64_t x);  // log() at atc :241-262
void atc_init(AtcState& s, const AtcParams& p);
void atc_report(AtcState& s, const AtcParams& p, uint64_t wait);  // do_vcrd_op, :210-229
void atc_update(AtcState& s, const AtcParams& p);                  // update_time_slice, :291-460

}  // namespace gpbs
