// Native gang coordinator: the per-rank epoch loop of cross-GPU gang windows
// (pbs_amd/parallel/gang.py documents the protocol)
// as a C++ thread bound to this GPU's engine, on the shm transport
// (gang_shm.cpp).  The Python coordinator ran the same loop under the GIL next
// to the bench's tenant threads; here no epoch waits on the interpreter.
//
// Per epoch, every member rank contributes one int64 vector
//   [demand(t) for t] [-wait_us(t) for t] [atc_local, keep_going, t_prev, -t_prev]
// and takes the element-wise MIN over the members' rows: demand on every rank,
// the worst rank's K10 wait, the node-wide ATC minimum (the global minimum
// sched_credit_atc.c applies every period, X:xen/common/sched_credit_atc.c),
// a collective stop, and the spread of the previous epoch's return time.  The
// window decision is a pure function of (epoch, reduced vector), so all ranks
// agree without a second message.  Every `metric_every` epochs a second
// exchange SUMs the metric tenants' last-period counter deltas: node-wide
// per-tenant metrics, the master's cross-CPU pmc gather of
// csched_dom_metric_update (X:xen/common/sched_credit.c:416-424) without a
// master.  A missed deadline records GANG_TIMEOUT and either re-forms the view
// among the survivors (gpbs_gang_shm_reform) or degrades to local scheduling.
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "gpbs/gpbs.h"

extern "C" {
int gpbs_gang_shm_allgather(void* h, uint64_t epoch, const int64_t* in, int64_t* out, int64_t deadline_ns);
int gpbs_gang_shm_reform(void* h, int64_t join_ns, int64_t deadline_ns, uint64_t* members, uint64_t* base_epoch);
}

namespace {

constexpr int64_t kNoAtc = 1ll << 30;  // MIN-neutral "no ATC pool on this rank"
constexpr int kFavour = 1, kExclude = 2, kNone = 0;
constexpr size_t kHistory = 8192;
constexpr size_t kLatKeep = 4096;

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000ll + ts.tv_nsec;
}

void sleep_ns(int64_t ns) {
  if (ns <= 0) return;
  timespec ts{(time_t)(ns / 1000000000ll), (long)(ns % 1000000000ll)};
  nanosleep(&ts, nullptr);
}

struct Metric {
  int64_t v[4] = {0, 0, 0, 0};  // inst, cycles, l2 refs, l2 misses
};

struct Coord {
  gpbs_engine_t* e = nullptr;
  void* shm = nullptr;
  gpbs_gang_cfg_t cfg{};
  int world = 1, nvals = 0;
  uint64_t seq = 0, members = 0;
  std::thread th;
  std::atomic<bool> want_stop{false};
  std::atomic<bool> finished{false};
  std::mutex mu;  // guards everything below against readers (stats, history)
  uint64_t epoch = 0;
  std::vector<int32_t> state, gang_on, on_since;
  std::vector<int64_t> ewma_us, wait_prev;
  std::vector<bool> wait_seen;
  std::deque<std::pair<uint64_t, std::vector<int32_t>>> history;
  std::deque<int64_t> lat, skew;
  std::vector<Metric> node, totals;
  int64_t timeouts = 0, reforms = 0, metric_syncs = 0, switches = 0, atc_global = 0;
  int degraded = 0, error = 0;
};

// ------------------------------------------------------------------ engine
bool demand(Coord* c, int t) {
  gpbs_tenant_info_t ti;
  if (gpbs_tenant_info(c->e, t, &ti)) return false;
  for (int k = 0; k < ti.nslots; ++k) {
    gpbs_slot_info_t si;
    const int s = gpbs_slot_id(c->e, t, k);
    if (s < 0 || gpbs_slot_info(c->e, s, &si)) continue;
    if (si.is_running || si.runstate <= 1) return true;
  }
  return false;
}

int64_t local_wait_us(Coord* c, int i) {
  gpbs_tenant_info_t ti;
  if (gpbs_tenant_info(c->e, c->cfg.tenants[i], &ti)) return 0;
  const int64_t cur = (int64_t)ti.spin_latency;
  const int64_t prev = c->wait_seen[i] ? c->wait_prev[i] : cur;
  c->wait_prev[i] = cur;
  c->wait_seen[i] = true;
  return std::max<int64_t>(0, cur - prev) / 1000;
}

int64_t atc_local(Coord* c) {
  if (c->cfg.atc_pool < 0) return kNoAtc;
  const int v = gpbs_atc_sync(c->e, c->cfg.atc_pool, 0);
  return v > 0 ? v : kNoAtc;
}

// ------------------------------------------------------------- transport
// why: 0 ok, 1 timeout, 2 excluded, 3 a newer view is forming
int gather(Coord* c, const std::vector<int64_t>& in, std::vector<int64_t>& rows, int64_t deadline, int* why) {
  std::vector<int64_t> v(in);
  v.resize(c->nvals, 0);
  rows.assign((size_t)c->nvals * c->world, 0);
  const int rc = gpbs_gang_shm_allgather(c->shm, ++c->seq, v.data(), rows.data(), deadline);
  *why = rc == 0 ? 0 : rc == -110 ? 1 : rc == -116 ? 2 : rc == -117 ? 3 : -1;
  if (*why < 0) c->error = rc;
  return rc;
}

template <class Op>
bool reduce(Coord* c, const std::vector<int64_t>& in, std::vector<int64_t>& out, int64_t deadline, int* why, Op op) {
  std::vector<int64_t> rows;
  if (gather(c, in, rows, deadline, why)) return false;
  out.assign(in.size(), 0);
  bool first = true;
  for (int r = 0; r < c->world; ++r) {
    if (!((c->members >> r) & 1)) continue;
    for (size_t j = 0; j < in.size(); ++j) {
      const int64_t x = rows[(size_t)r * c->nvals + j];
      out[j] = first ? x : op(out[j], x);
    }
    first = false;
  }
  return true;
}

void range_push(Coord* c, uint64_t epoch) {
  if (!c->cfg.roctx_push) return;
  char name[64];
  snprintf(name, sizeof name, "gpbs:gang_epoch %llu", (unsigned long long)epoch);
  c->cfg.roctx_push(name);
}

void range_pop(Coord* c) {
  if (c->cfg.roctx_pop) c->cfg.roctx_pop();
}

void on_timeout(Coord* c, int64_t waited_ns) {
  {
    std::lock_guard<std::mutex> g(c->mu);
    ++c->timeouts;
    c->degraded = 1;
  }
  gpbs_gang_timeout(c->e, (uint32_t)c->epoch, (uint32_t)c->cfg.rank, (uint32_t)(waited_ns / 1000));
}

bool reform(Coord* c) {
  if (!c->cfg.reform) return false;
  uint64_t m = 0, base = 0;
  if (c->cfg.roctx_push) c->cfg.roctx_push("gpbs:gang_reform");
  const int rc = gpbs_gang_shm_reform(c->shm, c->cfg.join_ns, mono_ns() + c->cfg.join_ns + c->cfg.deadline_ns, &m,
                                      &base);
  range_pop(c);
  if (rc) return false;
  std::lock_guard<std::mutex> g(c->mu);
  ++c->reforms;
  c->degraded = 0;
  c->members = m;
  c->seq = base - 1;
  c->epoch = base;  // decisions are a function of the epoch: the same on every member
  return true;
}

// --------------------------------------------------------------- decision
void update_gang_on(Coord* c, uint64_t epoch, const int64_t* max_wait_us) {
  const double on_us = c->cfg.wait_on_frac * (double)c->cfg.epoch_ns / 1e3;
  for (int i = 0; i < c->cfg.ntenants; ++i) {
    const int64_t ew = (3 * c->ewma_us[i] + max_wait_us[i]) / 4;  // waits are >= 0: floor division
    c->ewma_us[i] = ew;
    if (!c->gang_on[i] && (double)ew >= on_us) {
      c->gang_on[i] = 1;
      c->on_since[i] = (int32_t)epoch;
      ++c->switches;
    } else if (c->gang_on[i] && (int64_t)epoch - c->on_since[i] >= c->cfg.wait_hold_epochs && (double)ew < on_us / 4) {
      c->gang_on[i] = 0;
      ++c->switches;
    }
  }
}

std::vector<int32_t> decide(Coord* c, uint64_t epoch, const int64_t* demand_all) {
  const int nt = c->cfg.ntenants;
  std::vector<int32_t> out(nt, kNone);
  std::vector<int> eligible;
  for (int i = 0; i < nt; ++i)
    if (demand_all[i] && c->gang_on[i]) eligible.push_back(i);
  if (eligible.empty()) return out;
  const int period = 8;
  // round-half-even, as gang.py's round(): share 0.5 -> 4 of 8 epochs
  const int slots = std::max(1, std::min(period, (int)std::nearbyint(c->cfg.share * period)));
  const int pos = (int)(epoch % period);
  const int winner = pos < slots ? eligible[(pos + epoch / period) % eligible.size()] : -1;
  for (int i : eligible) out[i] = i == winner ? kFavour : kExclude;
  return out;
}

// C11: SUM over ranks of each metric tenant's last-period deltas (node
// metrics) and of its CUMULATIVE counters (gpbs_tenant_vpmu: the node-wide
// run totals are exact, whatever the exchange cadence -- summing sampled
// last periods would count ~1 period in every metric_every epochs).
bool sync_metrics(Coord* c, int* why) {
  const int nm = c->cfg.nmetric;
  std::vector<int64_t> vals(8 * nm, 0);
  for (int i = 0; i < nm; ++i) {
    gpbs_tenant_info_t ti;
    uint64_t cum[4] = {0, 0, 0, 0};
    if (!gpbs_tenant_info(c->e, c->cfg.metric_tenants[i], &ti))
      for (int k = 0; k < 4; ++k) vals[4 * i + k] = (int64_t)ti.pmc[k];
    if (!gpbs_tenant_vpmu(c->e, c->cfg.metric_tenants[i], cum))
      for (int k = 0; k < 4; ++k) vals[4 * nm + 4 * i + k] = (int64_t)cum[k];
  }
  std::vector<int64_t> red;
  if (!reduce(c, vals, red, mono_ns() + c->cfg.deadline_ns, why, [](int64_t a, int64_t b) { return a + b; }))
    return false;
  std::lock_guard<std::mutex> g(c->mu);
  for (int i = 0; i < nm; ++i)
    for (int k = 0; k < 4; ++k) {
      c->node[i].v[k] = red[4 * i + k];
      c->totals[i].v[k] = red[4 * nm + 4 * i + k];
    }
  ++c->metric_syncs;
  return true;
}

// -------------------------------------------------------------------- loop
void loop(Coord* c) {
  const int nt = c->cfg.ntenants;
  int64_t t_prev = 0;
  auto fail = [&](int why, int64_t since) -> bool {  // true: carry on in a re-formed view
    if (why == 1) on_timeout(c, mono_ns() - since);
    if (reform(c)) return true;
    if (why != 1) on_timeout(c, mono_ns() - since);  // excluded for good: recorded like a missed deadline
    return false;
  };
  for (;;) {
    const int64_t hang = gpbs_fault_fire(c->e, "rank_hang");
    if (hang >= 0) sleep_ns(std::max<int64_t>(hang, 1) * 1000000ll);  // GPBS_FAULT rank_hang=ppm:ms
    const int64_t t0 = mono_ns();
    std::vector<int64_t> vec;
    for (int i = 0; i < nt; ++i) vec.push_back(demand(c, c->cfg.tenants[i]) ? 1 : 0);
    for (int i = 0; i < nt; ++i) vec.push_back(-local_wait_us(c, i));  // MIN of -w = -(max over ranks)
    vec.insert(vec.end(), {atc_local(c), c->want_stop.load() ? 0 : 1, t_prev, -t_prev});
    const int64_t dl = c->epoch ? c->cfg.deadline_ns : c->cfg.start_ns;  // the first absorbs start-up skew
    std::vector<int64_t> red;
    int why = 0;
    range_push(c, c->epoch);
    const int64_t tg = mono_ns();
    const bool ok = reduce(c, vec, red, t0 + dl, &why, [](int64_t a, int64_t b) { return std::min(a, b); });
    range_pop(c);
    const int64_t t1 = mono_ns();
    if (!ok) {
      if (why < 0 || !fail(why, t0)) break;
      continue;
    }
    t_prev = t1;
    const size_t n = red.size();
    {
      std::lock_guard<std::mutex> g(c->mu);
      c->lat.push_back(t1 - t0);
      if (red[n - 2] > 0) c->skew.push_back(-red[n - 1] - red[n - 2]);
      while (c->lat.size() > kLatKeep) c->lat.pop_front();
      while (c->skew.size() > kLatKeep) c->skew.pop_front();
    }
    if (!red[n - 3]) break;  // some rank asked to stop: every rank leaves at this epoch
    if (c->cfg.atc_pool >= 0 && red[n - 4] > 0 && red[n - 4] < kNoAtc) {
      c->atc_global = red[n - 4];
      gpbs_atc_sync(c->e, c->cfg.atc_pool, (int)red[n - 4]);
    }
    if (c->cfg.nmetric && c->epoch % (uint64_t)std::max(1, c->cfg.metric_every) == 0) {
      if (!sync_metrics(c, &why)) {
        if (why < 0 || !fail(why, t1)) break;
        continue;
      }
    }
    std::vector<int64_t> wmax(nt);
    for (int i = 0; i < nt; ++i) wmax[i] = -red[nt + i];
    std::vector<int32_t> dec;
    {
      std::lock_guard<std::mutex> g(c->mu);
      if (c->cfg.wait_driven) update_gang_on(c, c->epoch, wmax.data());
      dec = decide(c, c->epoch, red.data());
    }
    const int64_t until = gpbs_now(c->e) + c->cfg.epoch_ns + c->cfg.slack_ns;
    for (int i = 0; i < nt; ++i) gpbs_gang_set(c->e, c->cfg.tenants[i], dec[i], until);
    {
      std::lock_guard<std::mutex> g(c->mu);
      c->state = dec;
      c->history.emplace_back(c->epoch, dec);
      while (c->history.size() > kHistory) c->history.pop_front();
      ++c->epoch;
    }
    sleep_ns(c->cfg.epoch_ns - (mono_ns() - t1));
  }
  for (int i = 0; i < nt; ++i) gpbs_gang_set(c->e, c->cfg.tenants[i], kNone, 0);
  c->finished.store(true, std::memory_order_release);
}

int64_t pct(std::vector<int64_t> v, double q) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(q * v.size()))];
}

}  // namespace

extern "C" {

void* gpbs_gang_coord_start(gpbs_engine_t* e, void* shm, int world, int nvals, const gpbs_gang_cfg_t* cfg) {
  if (!e || !shm || !cfg || cfg->ntenants < 0 || cfg->ntenants > GPBS_GANG_MAX_TENANTS || cfg->nmetric < 0 ||
      cfg->nmetric > GPBS_GANG_MAX_TENANTS || world < 1 || world > 64 || cfg->epoch_ns <= 0)
    return nullptr;
  if (nvals < 2 * cfg->ntenants + 4 || nvals < 8 * cfg->nmetric) return nullptr;
  auto* c = new Coord;
  c->e = e;
  c->shm = shm;
  c->cfg = *cfg;
  c->world = world;
  c->nvals = nvals;
  c->members = world >= 64 ? ~0ull : ((1ull << world) - 1);
  const int nt = cfg->ntenants;
  c->state.assign(nt, kNone);
  c->gang_on.assign(nt, cfg->wait_driven ? 0 : 1);
  c->on_since.assign(nt, 0);
  c->ewma_us.assign(nt, 0);
  c->wait_prev.assign(nt, 0);
  c->wait_seen.assign(nt, false);
  c->node.assign(cfg->nmetric, Metric{});
  c->totals.assign(cfg->nmetric, Metric{});
  c->th = std::thread(loop, c);
  return c;
}

// Ask every rank to stop (collective: the loop leaves at the first epoch in
// which some rank contributed keep_going = 0) and wait up to timeout_ns.
// 0 when the loop has finished (thread joined), -110 otherwise.
int gpbs_gang_coord_stop(void* h, int64_t timeout_ns) {
  auto* c = (Coord*)h;
  if (!c) return -22;
  c->want_stop = true;
  // poll (no condition variable: libstdc++'s timed wait goes through
  // pthread_cond_clockwait, which ThreadSanitizer does not model)
  const int64_t until = mono_ns() + timeout_ns;
  while (!c->finished.load(std::memory_order_acquire)) {
    if (mono_ns() > until) return -110;
    sleep_ns(200000);
  }
  if (c->th.joinable()) c->th.join();
  return 0;
}

int gpbs_gang_coord_running(void* h) {
  auto* c = (Coord*)h;
  return c && !c->finished.load() ? 1 : 0;
}

int gpbs_gang_coord_stats(void* h, gpbs_gang_stats_t* o) {
  auto* c = (Coord*)h;
  if (!c || !o) return -22;
  std::lock_guard<std::mutex> g(c->mu);
  std::vector<int64_t> lat(c->lat.begin(), c->lat.end()), skew(c->skew.begin(), c->skew.end());
  std::memset(o, 0, sizeof *o);
  o->epochs = (int64_t)c->epoch;
  o->sync_p50_ns = pct(lat, 0.5);
  o->sync_p99_ns = pct(lat, 0.99);
  o->sync_max_ns = lat.empty() ? 0 : *std::max_element(lat.begin(), lat.end());
  o->skew_p50_ns = pct(skew, 0.5);
  o->skew_max_ns = skew.empty() ? 0 : *std::max_element(skew.begin(), skew.end());
  o->timeouts = c->timeouts;
  o->degraded = c->degraded;
  o->reforms = c->reforms;
  o->members = (int64_t)c->members;
  o->atc_global_us = c->atc_global;
  o->metric_syncs = c->metric_syncs;
  o->gang_switches = c->switches;
  o->error = c->error;
  o->finished = c->finished.load() ? 1 : 0;
  return 0;
}

// Per gang tenant i: current window state, gang_on, wait EWMA (us).
int gpbs_gang_coord_tenant(void* h, int i, int64_t out[3]) {
  auto* c = (Coord*)h;
  if (!c || i < 0 || i >= c->cfg.ntenants) return -22;
  std::lock_guard<std::mutex> g(c->mu);
  out[0] = c->state[i];
  out[1] = c->gang_on[i];
  out[2] = c->ewma_us[i];
  return 0;
}

// Per metric tenant i: the last node-wide SUM and the run totals
// (inst, cycles, l2 refs, l2 misses).
int gpbs_gang_coord_metrics(void* h, int i, int64_t last[4], int64_t totals[4]) {
  auto* c = (Coord*)h;
  if (!c || i < 0 || i >= c->cfg.nmetric) return -22;
  std::lock_guard<std::mutex> g(c->mu);
  for (int k = 0; k < 4; ++k) {
    last[k] = c->node[i].v[k];
    totals[k] = c->totals[i].v[k];
  }
  return 0;
}

// The last <= max decisions: epochs[j], states[j * ntenants + i].  Returns the count.
int gpbs_gang_coord_history(void* h, int64_t* epochs, int32_t* states, int max) {
  auto* c = (Coord*)h;
  if (!c || max < 0) return -22;
  std::lock_guard<std::mutex> g(c->mu);
  const int n = (int)std::min<size_t>((size_t)max, c->history.size());
  const size_t first = c->history.size() - n;
  for (int j = 0; j < n; ++j) {
    const auto& hs = c->history[first + j];
    if (epochs) epochs[j] = (int64_t)hs.first;
    if (states) std::memcpy(states + (size_t)j * c->cfg.ntenants, hs.second.data(), sizeof(int32_t) * c->cfg.ntenants);
  }
  return n;
}

// Joins the loop (stop first: a running loop only leaves at a collective stop
// or a failure) and frees the coordinator.  The shm region stays the caller's.
void gpbs_gang_coord_destroy(void* h) {
  auto* c = (Coord*)h;
  if (!c) return;
  c->want_stop = true;
  if (c->th.joinable()) c->th.join();
  delete c;
}

}  // extern "C"
