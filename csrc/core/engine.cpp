// Generic scheduling framework.  Behavior parity references:
//   schedule()            X:xen/common/schedule.c:1082-1185
//   vcpu_wake/sleep       X:xen/common/schedule.c:331-380
//   vcpu_migrate          X:xen/common/schedule.c:404-470
//   context_saved         X:xen/common/schedule.c:1187-1201
//   cpupool ops           X:xen/common/cpupool.c:118-453
//   keyhandlers r/q/z     X:xen/common/cpupool.c:604-646, X:xen/common/keyhandler.c:233-300,421-426
#include "engine.h"

#include <sys/prctl.h>
#include <time.h>

#include <algorithm>
#include <cinttypes>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <tuple>

namespace gpbs {

namespace {
int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000ll + ts.tv_nsec;
}
std::string fmt(const char* f, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}
}  // namespace

Engine::Engine(const gpbs_boot_params_t& p) : boot(p) {
  std::memcpy(&adapt_params, &p.adapt, sizeof(adapt_params));
  std::memcpy(&atc_params, &p.atc, sizeof(atc_params));
  size_t cap = 1;
  while (cap < (size_t)std::max(1024, p.trace_capacity)) cap <<= 1;
  trace = std::make_unique<TraceRing>(cap);
  if (boot.sim_clock) sim_now = 0;
  pool_create("Pool-0", boot.sched);
  if (boot.coschedule >= 2) {
    class_timer_ = timer_init([this](int64_t n) { classify_tick(n); });
    timer_set(class_timer_, now() + (int64_t)std::max(100, boot.class_period_us) * 1000);
  }
  if (boot.heartbeat_timeout_us > 0) {
    hb_timer_ = timer_init([this](int64_t n) { heartbeat_check(n); });
    timer_set(hb_timer_, now() + (int64_t)boot.heartbeat_timeout_us * 1000 / 2);
  }
}

Engine::~Engine() {
  stop();
  ApiLock g(this);
  for (auto& p : pools)
    if (p && p->sched) p->sched->deinit();
}

int64_t Engine::now() const { return boot.sim_clock ? sim_now : mono_ns(); }

// ------------------------------------------------------------------ timers -

int Engine::timer_init(std::function<void(int64_t)> fn) {
  int id;
  if (!free_timers_.empty()) {
    id = free_timers_.back();
    free_timers_.pop_back();
  } else {
    id = (int)timers_.size();
    timers_.emplace_back();
  }
  TimerEnt& t = timers_[id];
  t.fn = std::move(fn);
  t.gen++;
  t.armed = false;
  t.alive = true;
  return id;
}

void Engine::timer_set(int id, int64_t when) {
  TimerEnt& t = timers_[id];
  if (!t.alive) return;
  t.gen++;
  t.armed = true;
  t.when = when;
  heap_.push(HeapEnt{when, seq_++, id, t.gen});
}

void Engine::timer_stop(int id) {
  if (id < 0) return;
  TimerEnt& t = timers_[id];
  t.armed = false;
  t.gen++;
}

void Engine::timer_kill(int id) {
  if (id < 0) return;
  TimerEnt& t = timers_[id];
  t.armed = false;
  t.alive = false;
  t.gen++;
  t.fn = nullptr;
  free_timers_.push_back(id);
}

bool Engine::timer_armed(int id) const { return id >= 0 && timers_[id].alive && timers_[id].armed; }

int64_t Engine::next_deadline() const {
  auto& h = const_cast<decltype(heap_)&>(heap_);
  while (!h.empty()) {
    const HeapEnt& e = h.top();
    const TimerEnt& t = timers_[e.id];
    if (t.alive && t.armed && t.gen == e.gen) return e.when;
    h.pop();
  }
  return INT64_MAX;
}

void Engine::run_due(int64_t n) {
  while (!heap_.empty() && heap_.top().when <= n) {
    HeapEnt e = heap_.top();
    heap_.pop();
    TimerEnt& t = timers_[e.id];
    if (!t.alive || !t.armed || t.gen != e.gen) continue;
    if (!e.jittered && fault(F_TIMER_JITTER)) {  // fire late, once
      e.when += std::max<int64_t>(1, fault_param[F_TIMER_JITTER]) * 1000;
      e.jittered = true;
      heap_.push(e);
      continue;
    }
    t.armed = false;
    int64_t tn = n;
    if (boot.sim_clock) {
      sim_now = e.when;
      tn = e.when;
    }
    auto fn = t.fn;  // the handler may re-arm or kill its own timer
    fn(tn);
    process_softirqs();
  }
  if (boot.sim_clock && n > sim_now) sim_now = n;
  process_softirqs();
  flush_actuation();
}

void Engine::raise_softirq(int part) {
  if (part >= 0 && part < (int)parts.size()) parts[part]->softirq = true;
}

void Engine::process_softirqs() {
  if (in_softirq_) return;
  in_softirq_ = true;
  for (;;) {
    bool any = false;
    for (auto& p : parts) {
      if (p->softirq) {
        p->softirq = false;
        any = true;
        if (p->pool >= 0) schedule(p->id);
      }
    }
    if (!any) break;
  }
  in_softirq_ = false;
}

void Engine::flush_actuation() {
  if (dirty_actuation && fault(F_ACTUATE_DELAY)) return;  // held back: applied with the next batch
  if (dirty_actuation && actuator_ops.on_flush) actuator_ops.on_flush(actuator_ops.user, now());
  dirty_actuation = false;
}

int Engine::fault_parse(const char* spec) {
  static const char* names[F_NKIND] = {"counter_drop", "counter_reset", "heartbeat_drop", "actuate_delay",
                                       "timer_jitter", "rank_hang", "torn_page"};
  if (!spec) return 0;
  int n = 0;
  std::string s(spec);
  size_t pos = 0;
  while (pos < s.size()) {
    size_t end = s.find(',', pos);
    if (end == std::string::npos) end = s.size();
    const std::string item = s.substr(pos, end - pos);
    pos = end + 1;
    const size_t eq = item.find('=');
    if (eq == std::string::npos) continue;
    const std::string key = item.substr(0, eq);
    const std::string val = item.substr(eq + 1);
    if (key == "seed") {
      fault_rng = std::strtoull(val.c_str(), nullptr, 0) | 1ull;
      continue;
    }
    for (int k = 0; k < F_NKIND; ++k)
      if (key == names[k]) {
        fault_ppm[k] = (uint32_t)std::min<unsigned long>(1000000ul, std::strtoul(val.c_str(), nullptr, 0));
        const size_t colon = val.find(':');
        if (colon != std::string::npos) fault_param[k] = std::strtoll(val.c_str() + colon + 1, nullptr, 0);
        ++n;
      }
  }
  if (n) printk(fmt("(GPBS) fault injection armed: %s\n", spec));
  return n;
}

// --------------------------------------------------------------- lifecycle -

int Engine::partition_add(int gpu, int xcd, int ctx) {
  if ((int)parts.size() >= kMaxPartitions) return GPBS_ENOSPC;
  auto p = std::make_unique<Partition>();
  p->id = (int)parts.size();
  p->gpu = gpu;
  p->xcd = xcd;
  p->ctx = ctx;
  auto idle = std::make_unique<Slot>();
  idle->id = (int)slots.size();
  idle->tenant = -1;
  idle->index = p->id;
  idle->processor = p->id;
  idle->affinity = Mask::of(p->id);
  idle->is_running = true;
  idle->rs = RS_RUNNING;
  idle->rs_entry = now();
  p->idle_slot = idle->id;
  p->curr = idle->id;
  const int pid = p->id;
  p->s_timer = timer_init([this, pid](int64_t) {  // s_timer_fn
    perfc.incr(PC_sched_irq);
    raise_softirq(pid);
  });
  slots.push_back(std::move(idle));
  parts.push_back(std::move(p));
  return pid;
}

int Engine::pool_create(const std::string& name, const std::string& sched) {
  for (auto& p : pools)
    if (p && p->name == name) return GPBS_EEXIST;
  auto pl = std::make_unique<Pool>();
  pl->id = (int)pools.size();
  pl->name = name;
  pl->sched_name = sched.empty() ? std::string(boot.sched) : sched;
  pl->sched = make_scheduler(pl->sched_name, *this, pl->id);
  if (!pl->sched) return GPBS_EINVAL;
  int rc = pl->sched->init();
  if (rc) return rc;
  int id = pl->id;
  pools.push_back(std::move(pl));
  emit(TRC_POOL, 0, id, 1, 0);
  return id;
}

int Engine::pool_destroy(int id) {
  Pool* pl = pool(id);
  if (!pl || id == 0) return GPBS_EINVAL;  // Pool-0 cannot be destroyed
  for (auto& t : tenants)
    if (t && t->alive && t->pool == id) return GPBS_EBUSY;
  if (!pl->cpus.empty()) return GPBS_EBUSY;  // cpupool_destroy requires no cpus
  pl->sched->deinit();
  pools[id].reset();
  emit(TRC_POOL, 0, id, 2, 0);
  return GPBS_OK;
}

int Engine::pool_assign(int id, int part) {
  Pool* pl = pool(id);
  if (!pl || part < 0 || part >= (int)parts.size()) return GPBS_EINVAL;
  Partition& P = *parts[part];
  if (P.pool >= 0) return GPBS_EBUSY;
  P.pool = id;
  pl->cpus.set(part);
  Slot& idle = *slots[P.idle_slot];
  pl->sched->alloc_vdata(idle);
  pl->sched->alloc_pdata(part);
  // Parked slots of this pool waiting for any partition can now run here.
  for (auto& s : slots) {
    if (!s || s->is_idle()) continue;
    Tenant* t = tenant(s->tenant);
    if (!t || t->pool != id) continue;
    if (!pl->cpus.test(s->processor)) {
      s->processor = part;
    }
  }
  raise_softirq(part);
  process_softirqs();
  emit(TRC_POOL, part, id, 3, part);
  return GPBS_OK;
}

int Engine::pool_unassign(int id, int part) {
  Pool* pl = pool(id);
  if (!pl || part < 0 || part >= (int)parts.size() || parts[part]->pool != id) return GPBS_EINVAL;
  bool has_tenants = false;
  for (auto& t : tenants)
    if (t && t->alive && t->pool == id) has_tenants = true;
  if (pl->cpus.weight() == 1 && has_tenants) return GPBS_EBUSY;  // last cpu of a busy pool
  Partition& P = *parts[part];
  pl->cpus.clear(part);
  // Evacuate: the running slot and every queued slot move to remaining cpus.
  std::vector<int> movers;
  for (auto& s : slots)
    if (s && !s->is_idle() && s->processor == part) movers.push_back(s->id);
  for (int sid : movers) {
    Slot& v = *slots[sid];
    v.pause_flags |= VPF_MIGRATING;
    vcpu_sleep_nosync(v);
  }
  // Deschedule whatever is running, then switch the cpu to its idle slot.
  if (P.curr != P.idle_slot) {
    raise_softirq(part);
    process_softirqs();
  }
  pl->sched->free_pdata(part);
  timer_stop(P.s_timer);
  P.pool = -1;
  for (int sid : movers) {
    Slot& v = *slots[sid];
    if (v.is_running) continue;  // handled by context_saved
    if (v.pause_flags & VPF_MIGRATING) vcpu_migrate(v);
  }
  // Affinity masks referencing the removed cpu stay valid for other cpus.
  process_softirqs();
  emit(TRC_POOL, part, id, 4, part);
  return GPBS_OK;
}

int Engine::tenant_create(const std::string& name, int poolid, int nslots, int weight, int cap) {
  Pool* pl = pool(poolid);
  if (!pl || nslots <= 0 || nslots > kMaxPartitions) return GPBS_EINVAL;
  if (weight != -1 && (weight < 1 || weight > GPBS_WEIGHT_MAX)) return GPBS_ERANGE;
  if (cap != -1 && (cap < 0 || cap > 100 * nslots)) return GPBS_ERANGE;
  for (auto& t : tenants)
    if (t && t->alive && t->name == name) return GPBS_EEXIST;
  auto T = std::make_unique<Tenant>();
  T->id = (int)tenants.size();
  T->name = name;
  T->pool = poolid;
  T->last_heartbeat = now();
  tenants.push_back(std::move(T));
  Tenant& d = *tenants.back();
  int rc = pl->sched->init_domain(d);
  if (rc) {
    tenants.pop_back();
    return rc;
  }
  perfc.incr(PC_dom_init);
  // Initial placement: default_vcpu0_location (X:xen/common/domctl.c:167-214)
  // puts vCPU 0 on the least-populated CPU (ties: highest-numbered) and
  // cycles the rest from there (:566-569).  gpbs applies the least-populated
  // rule to every slot, preferring XCDs the tenant does not occupy yet: the
  // cycle stacks slots of different tenants on one partition while another
  // idles, which schedulers without load balancing (sedf, static) never undo.
  std::vector<int> cnt(parts.size(), 0);
  for (auto& s : slots)
    if (s && !s->is_idle() && !(s->pause_flags & VPF_DOWN) && s->processor < (int)cnt.size()) cnt[s->processor]++;
  std::vector<int> mine;  // partitions holding this tenant's slots so far
  auto place = [&]() {
    int best = pl->cpus.empty() ? 0 : pl->cpus.first(), bkey = INT32_MAX;
    for (int c = pl->cpus.first(); c >= 0; c = pl->cpus.next(c + 1)) {
      int same_xcd = 0;
      for (int m : mine) same_xcd += parts[m]->gpu == parts[c]->gpu && parts[m]->xcd == parts[c]->xcd;
      const int key = cnt[c] * 1024 + same_xcd;
      if (key <= bkey) {
        bkey = key;
        best = c;
      }
    }
    return best;
  };
  for (int i = 0; i < nslots; ++i) {
    auto s = std::make_unique<Slot>();
    s->id = (int)slots.size();
    s->tenant = d.id;
    s->index = i;
    const int cpu = place();
    cnt[cpu]++;
    mine.push_back(cpu);
    s->processor = cpu;
    s->affinity = Mask::all(kMaxPartitions);  // setall (schedule.c:201)
    s->pause_flags = VPF_BLOCKED;             // no work yet
    s->rs = RS_BLOCKED;
    s->rs_entry = now();
    d.slots.push_back(s->id);
    Slot& v = *s;
    slots.push_back(std::move(s));
    pl->sched->alloc_vdata(v);
    pl->sched->insert_vcpu(v);
    perfc.incr(PC_vcpu_init);
  }
  int w = weight, c = cap;
  if (w != -1 || c != -1) pl->sched->adjust(d, true, &w, &c);
  return d.id;
}

int Engine::tenant_destroy(int tid) {
  Tenant* d = tenant(tid);
  if (!d || !d->alive) return GPBS_ENOENT;
  Scheduler* S = sched_of_tenant(tid);
  for (int sid : d->slots) {
    Slot& v = *slots[sid];
    v.pause_flags |= VPF_BLOCKED;
    vcpu_sleep_nosync(v);
  }
  process_softirqs();
  for (int sid : d->slots) {
    Slot& v = *slots[sid];
    S->remove_vcpu(v);
    perfc.incr(PC_vcpu_destroy);
    v.priv.reset();
  }
  S->destroy_domain(*d);
  perfc.incr(PC_dom_destroy);
  watchdog_kill(*d);  // watchdog_domain_destroy
  d->alive = false;
  d->priv.reset();
  for (int sid : d->slots) slots[sid].reset();
  d->slots.clear();
  flush_actuation();
  return GPBS_OK;
}

int Engine::tenant_move(int tid, int newpool) {
  Tenant* d = tenant(tid);
  Pool* np = pool(newpool);
  if (!d || !d->alive || !np) return GPBS_EINVAL;
  if (d->pool == newpool) return GPBS_OK;
  if (np->cpus.empty()) return GPBS_EINVAL;
  Scheduler* S = sched_of_tenant(tid);
  int w = -1, c = -1;
  S->adjust(*d, false, &w, &c);
  std::vector<bool> was_blocked;
  for (int sid : d->slots) {
    Slot& v = *slots[sid];
    was_blocked.push_back(v.pause_flags & VPF_BLOCKED);
    v.pause_flags |= VPF_BLOCKED;
    vcpu_sleep_nosync(v);
  }
  process_softirqs();
  for (int sid : d->slots) {
    S->remove_vcpu(*slots[sid]);
    slots[sid]->priv.reset();
  }
  S->destroy_domain(*d);
  d->priv.reset();
  d->pool = newpool;
  // Q4 fix: full init_domain (PBS state re-initialised, not just domdata).
  np->sched->init_domain(*d);
  int cpu = np->cpus.first();
  for (size_t i = 0; i < d->slots.size(); ++i) {
    Slot& v = *slots[d->slots[i]];
    v.processor = cpu;
    v.affinity = Mask::all(kMaxPartitions);
    np->sched->alloc_vdata(v);
    np->sched->insert_vcpu(v);
    cpu = np->cpus.cycle(cpu);
  }
  np->sched->adjust(*d, true, &w, &c);
  for (size_t i = 0; i < d->slots.size(); ++i)
    if (!was_blocked[i]) vcpu_unblock(*slots[d->slots[i]]);
  process_softirqs();
  flush_actuation();
  return GPBS_OK;
}

int Engine::tenant_set_nslots(int tid, int n) {
  Tenant* d = tenant(tid);
  if (!d || !d->alive || n < 1 || n > kMaxPartitions) return GPBS_EINVAL;
  Scheduler* S = sched_of_tenant(tid);
  Pool* pl = pool(d->pool);
  while ((int)d->slots.size() < n) {  // grow (max_vcpus)
    auto s = std::make_unique<Slot>();
    s->id = (int)slots.size();
    s->tenant = d->id;
    s->index = (int)d->slots.size();
    s->processor = pl->cpus.empty() ? 0 : pl->cpus.first();
    s->affinity = Mask::all(kMaxPartitions);
    s->pause_flags = VPF_BLOCKED;
    s->rs = RS_BLOCKED;
    s->rs_entry = now();
    d->slots.push_back(s->id);
    Slot& v = *s;
    slots.push_back(std::move(s));
    S->alloc_vdata(v);
    S->insert_vcpu(v);
  }
  for (size_t i = 0; i < d->slots.size(); ++i) {
    Slot& v = *slots[d->slots[i]];
    if ((int)i < n && (v.pause_flags & VPF_DOWN)) {
      v.pause_flags &= ~VPF_DOWN;
      vcpu_wake(v);
    } else if ((int)i >= n && !(v.pause_flags & VPF_DOWN)) {
      v.pause_flags |= VPF_DOWN;
      vcpu_sleep_nosync(v);
    }
  }
  process_softirqs();
  flush_actuation();
  return GPBS_OK;
}

Scheduler* Engine::sched_of_part(int part) {
  int p = parts[part]->pool;
  return p >= 0 && pools[p] ? pools[p]->sched.get() : nullptr;
}

Scheduler* Engine::sched_of_tenant(int t) {
  Tenant* d = tenant(t);
  return d && pools[d->pool] ? pools[d->pool]->sched.get() : nullptr;
}

// ------------------------------------------------------- generic vcpu ops --

bool Engine::runnable(const Slot& v) const {
  if (v.is_idle()) return true;
  if (v.pause_flags || v.pause_count) return false;
  const Tenant* d = tenants[v.tenant].get();
  return d && d->alive && d->pause_count == 0;
}

void Engine::runstate_change(Slot& v, Runstate rs, int64_t n) {
  if (n > v.rs_entry) v.rs_time[v.rs] += n - v.rs_entry;
  v.rs = rs;
  v.rs_entry = n;
}

void Engine::vcpu_wake(Slot& v) {
  if (runnable(v)) {
    // a wake is work: the class_budget presence test sees a tenant whose
    // requests are shorter than the class tick (an in-region latency tenant
    // is blocked at almost every tick; round 6 slo mix: it flapped between
    // present and absent, re-laying the region every ~10 ms)
    if (!v.is_idle() && tenants[v.tenant]->pause_count == 0) tenants[v.tenant]->last_busy = now();
    if (v.rs >= RS_BLOCKED) runstate_change(v, RS_RUNNABLE, now());
    if (Scheduler* S = sched_of_tenant(v.tenant)) {
      if (pools[tenants[v.tenant]->pool]->cpus.empty()) return;  // pool without cpus: stays queued later
      S->wake(v);
    }
  } else if (!(v.pause_flags & VPF_BLOCKED)) {
    if (v.rs == RS_BLOCKED) runstate_change(v, RS_OFFLINE, now());
  }
  uint32_t wv = 0, wc = 0;
  if (Scheduler* S = sched_of_tenant(v.tenant)) {
    wv = S->trace_word(v);
    wc = S->trace_word(*slots[parts[v.processor]->curr]);
  }
  emit(TRC_WAKE, v.processor, v.tenant, v.index, wv, wc);
}

void Engine::vcpu_sleep_nosync(Slot& v) {
  if (!runnable(v)) {
    if (v.rs == RS_RUNNABLE)
      runstate_change(v, (v.pause_flags & VPF_BLOCKED) ? RS_BLOCKED : RS_OFFLINE, now());
    if (Scheduler* S = sched_of_tenant(v.tenant)) S->sleep(v);
  }
  emit(TRC_SLEEP, v.processor, v.tenant, v.index, v.processor);
}

void Engine::vcpu_block(Slot& v) {
  if (v.pause_flags & VPF_BLOCKED) return;
  v.pause_flags |= VPF_BLOCKED;
  vcpu_sleep_nosync(v);
}

void Engine::vcpu_unblock(Slot& v) {
  if (!(v.pause_flags & VPF_BLOCKED)) return;
  v.pause_flags &= ~VPF_BLOCKED;
  vcpu_wake(v);
}

void Engine::vcpu_pause(Slot& v) {
  v.pause_count++;
  vcpu_sleep_nosync(v);
}

void Engine::vcpu_unpause(Slot& v) {
  if (v.pause_count > 0 && --v.pause_count == 0) vcpu_wake(v);
}

void Engine::vcpu_migrate(Slot& v) {
  Scheduler* S = sched_of_tenant(v.tenant);
  if (!S) return;
  Pool* pl = pools[tenants[v.tenant]->pool].get();
  int old = v.processor;
  v.pause_flags &= ~VPF_MIGRATING;
  if (pl->cpus.empty()) return;
  if (!pl->cpus.test(v.processor)) v.processor = pl->cpus.first();
  int nc;
  if (v.home >= 0 && pl->cpus.test(v.home) && v.affinity.test(v.home)) {
    nc = v.home;  // class placement spreads a tenant's slots one per partition
    v.homed_at = now();
  } else
    nc = S->pick_cpu(v);
  v.home = -1;
  v.processor = nc;
  if (old != nc) emit(TRC_MIGRATE, nc, v.tenant, v.index, old, nc);
  vcpu_wake(v);
}

void Engine::pmu_refresh(Slot& v) {
  if (v.is_idle()) return;
  if (fault(F_COUNTER_RESET)) {  // PMU reset under the scheduler (Q5)
    for (int i = 0; i < kNumPmc; ++i) v.pmc[i] = 0;
    return;
  }
  if (fault(F_COUNTER_DROP) || !counter_ops.slot_refresh) return;
  counter_ops.slot_refresh(counter_ops.user, v.id, v.tenant, v.processor, v.pmc);
}

void Engine::schedule(int part) {
  Partition& P = *parts[part];
  Scheduler* S = sched_of_part(part);
  if (!S) return;
  const int64_t n = now();
  perfc.incr(PC_sched_run);
  Slot& prev = *slots[P.curr];
  timer_stop(P.s_timer);
  TaskSlice ts = S->do_schedule(part, n);
  Slot& next = *slots[ts.slot];
  P.curr = next.id;
  if (ts.time_ns >= 0) {
    int64_t when = n + ts.time_ns;
    if (boot.quantum_align_us > 0) {  // batch switches of all partitions onto a common grid
      const int64_t a = (int64_t)boot.quantum_align_us * 1000;
      when = (when + a - 1) / a * a;
    }
    timer_set(P.s_timer, when);
  }
  if (&prev == &next) return;  // continue_running
  const int32_t q_us = ts.time_ns >= 0 ? (int32_t)(ts.time_ns / 1000) : -1;
  emit(TRC_SWITCH, part, (uint32_t)prev.tenant, (uint32_t)next.tenant, (uint32_t)q_us);
  runstate_change(prev,
                  (prev.pause_flags & VPF_BLOCKED) ? RS_BLOCKED : (runnable(prev) ? RS_RUNNABLE : RS_OFFLINE), n);
  prev.last_run_time = n;
  runstate_change(next, RS_RUNNING, n);
  next.is_running = true;
  perfc.incr(PC_sched_ctx);
  // context_switch: PMU save of prev (pmustate.c:87-111 / P4), count next.
  pmu_refresh(prev);
  if (!next.is_idle()) next.sched_count++;
  P.switches++;
  if (actuator_ops.on_switch) {
    actuator_ops.on_switch(actuator_ops.user, part, prev.tenant, next.tenant, next.is_idle() ? -1 : next.id, q_us, n);
    perfc.incr(PC_partition_switch);
  }
  dirty_actuation = true;
  context_saved(prev);
}

void Engine::context_saved(Slot& prev) {
  prev.is_running = false;
  if (Scheduler* S = sched_of_tenant(prev.tenant)) S->context_saved(prev);
  if (prev.pause_flags & VPF_MIGRATING) vcpu_migrate(prev);
}

// ------------------------------------------------- contention-class placement --
// gpbs extension (MI355X): the issue contexts of an XCD are typed.  Context 0
// hosts compute-bound (MFMA) tenants, context 1 memory-bound ones, so every
// XCD co-runs one of each (their waves use different pipes of the same CUs)
// while memory-bound tenants, which would only split HBM bandwidth, time-share
// their context under credit fairness and PBS's long cache-sensitive quanta.
// The class comes from the PBS counter rates, with two-tick hysteresis, and is
// a SOFT affinity (Xen 4.5 semantics): placement, cpu_pick and stealing prefer
// the class's partitions, but an idle partition of the other class may still
// steal a waiting slot (work conservation when a class runs dry), and the
// class tick sends such slots home once they stop running.
void Engine::send_home(Slot& v) {
  if (v.class_home < 0 || v.processor == v.class_home || !v.affinity.test(v.class_home)) return;
  v.home = v.class_home;
  v.pause_flags |= VPF_MIGRATING;
  vcpu_sleep_nosync(v);
  if (!v.is_running) vcpu_migrate(v);
}

void Engine::place_class(Slot& v, const Mask& m, int home) {
  v.soft = m;
  v.class_home = (home >= 0 && m.test(home)) ? home : -1;
  send_home(v);
}

void Engine::set_affinity(Slot& v, const Mask& m, int home) {
  v.affinity = m;
  v.home = (home >= 0 && m.test(home)) ? home : -1;
  if (!m.test(v.processor) || (v.home >= 0 && v.processor != v.home)) {
    v.pause_flags |= VPF_MIGRATING;
    vcpu_sleep_nosync(v);
    if (!v.is_running) vcpu_migrate(v);
  }
}

void Engine::place_tenant_class(Tenant& t, Pool& pl, int layout) {
  const int c = t.cls;
  // Class 0 (compute) lives on contexts [0, class_split) -- context 0 by
  // default; the memory class on every other context (with two contexts
  // per XCD: context 1).  In SE-exclusive mode (class_split 2 of 4) the
  // classes own shader engines {0,1} and {2,3} of every XCD.  A class alone
  // in the pool (layout = one bit) takes every context.
  const int split = std::max(1, boot.class_split);
  const bool alone = layout == (1 << c);
  Mask m;
  for (int p = pl.cpus.first(); p >= 0; p = pl.cpus.next(p + 1))
    if (alone || (c == 0 ? parts[p]->ctx < split : parts[p]->ctx >= split)) m.set(p);
  if (m.empty()) m = pl.cpus;
  // Slot k goes to the k-th partition of the class (cycling), ordered
  // context-major, so a tenant with one slot per XCD lands on every XCD
  // instead of wherever pick_cpu's cycle from its old processor would pile
  // them up.  Co-class tenants start where the previous one's slots end
  // (slot counts accumulated in id order): two 16-slot GEMMs on 32 SE
  // partitions take SEs {0,1} and {2,3}; two 8-slot memory tenants on the
  // 16 memory partitions one SE each; a class with more slots than
  // partitions (two 16-slot memory tenants: the time-shared variant) is
  // staggered by context instead.
  std::vector<int> order;
  for (int p = m.first(); p >= 0; p = m.next(p + 1)) order.push_back(p);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    return std::make_tuple(parts[a]->ctx, parts[a]->gpu, parts[a]->xcd) <
           std::make_tuple(parts[b]->ctx, parts[b]->gpu, parts[b]->xcd);
  });
  size_t rot = 0;
  for (auto& up : tenants)
    if (up && up->alive && up->priv && up->pool == pl.id && up->cls == c && up->id < t.id) rot += up->slots.size();
  if (rot + t.slots.size() > order.size() && !order.empty()) {
    // The class holds more slots than partitions (time-shared): stagger the
    // tenants by whole contexts, by id, so each partition's runqueue mixes
    // them (identical homes let one tenant's gang hold every partition).
    const int c0 = parts[order[0]]->ctx;
    size_t per = 0;
    while (per < order.size() && parts[order[per]]->ctx == c0) ++per;
    const size_t nc = order.size() / std::max<size_t>(per, 1);
    rot = nc > 1 ? (size_t)(t.id % (int)nc) * per : 0;
  }
  for (size_t k = 0; k < t.slots.size(); ++k)
    place_class(*slots[t.slots[k]], m, order.empty() ? -1 : order[(k + rot) % order.size()]);
  emit(TRC_CLASS, 0, t.id, (uint32_t)c, (uint32_t)m.weight());
}

// ------------------------------------------- demand-driven SE budgets ----
// class_budget (gpbs extension, SE-exclusive mode): instead of fixed class
// halves whose per-tenant share is whatever slot count the tenant was created
// with, every classified tenant that is PRESENT (a runnable slot now, or
// within present_us) gets a set of shader engines of every XCD, sized from
// the classes present -- the cpupool-resize analog of a credit scheduler's
// work conservation, at the granularity the hardware can confine:
//   * both classes present: compute owns contexts [0, class_split), memory
//     the rest; one class alone spans every context;
//   * a class region of r contexts with n <= r tenants is split into aligned
//     blocks (r = 4: one tenant 4, two 2+2, three 2+1+1, four 1 each; r = 2:
//     2, or 1+1) -- never a 3-SE set, which no class-half CU-masked stream
//     covers;
//   * n > r: every tenant of the region gets the whole region, staggered, and
//     credit time-shares it with PBS quanta (the class region is one gang).
// A busy tenant that is not classified yet is placed as memory class until
// its counters say otherwise.
// A tenant gets exactly one online slot per partition of its set; surplus
// slots go offline (VPF_DOWN, the vcpu-set path), so its share follows the
// layout instead of a creation-time slot count.  An absent tenant keeps its
// slots (blocked); it re-enters the layout at the first class tick after it
// has work again.  Reference analog: credit's idle-CPU stealing and tickling
// make the pCPUs a blocked domain leaves available to the others at once
// (X:xen/common/sched_credit.c:1559-1672); here that happens per class tick,
// in space.
void Engine::place_budget(Tenant& t, Pool& pl, uint32_t ctx_mask, int stagger, uint32_t xcd_mask) {
  Mask m;
  for (int p = pl.cpus.first(); p >= 0; p = pl.cpus.next(p + 1))
    if (((ctx_mask >> (parts[p]->ctx & 31)) & 1) && (!xcd_mask || ((xcd_mask >> (parts[p]->xcd & 31)) & 1))) m.set(p);
  std::vector<int> order;
  for (int p = m.first(); p >= 0; p = m.next(p + 1)) order.push_back(p);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    return std::make_tuple(parts[a]->ctx, parts[a]->gpu, parts[a]->xcd) <
           std::make_tuple(parts[b]->ctx, parts[b]->gpu, parts[b]->xcd);
  });
  const size_t online = std::min(order.size(), t.slots.size());
  for (size_t k = 0; k < t.slots.size(); ++k) {
    Slot& v = *slots[t.slots[k]];
    if (k < online) {
      if (v.pause_flags & VPF_DOWN) {
        v.pause_flags &= ~VPF_DOWN;
        v.home = order[(k + (size_t)stagger) % order.size()];
        v.soft = m;
        v.class_home = v.home;
        if (!v.is_running) {
          v.processor = v.home;  // an offline slot is on no runqueue: place it before it wakes
          v.home = -1;
        }
        vcpu_wake(v);
      } else {
        place_class(v, m, order[(k + (size_t)stagger) % order.size()]);
      }
    } else if (!(v.pause_flags & VPF_DOWN)) {
      v.pause_flags |= VPF_DOWN;
      v.class_home = -1;
      v.soft = Mask();
      vcpu_sleep_nosync(v);
    }
  }
  t.budget_ctx = ctx_mask | ((xcd_mask & 0xffu) << 8);
  emit(TRC_CLASS, 0, t.id, (uint32_t)t.cls, (uint32_t)m.weight());
}

// A tenant's budget as an explicit set of partitions (mem_split blocks): one
// online slot per partition, homes in context-major order.
void Engine::place_parts(Tenant& t, Pool& pl, const Mask& m) {
  std::vector<int> order;
  uint32_t ctxs = 0, xcds = 0;
  for (int p = m.first(); p >= 0; p = m.next(p + 1)) {
    order.push_back(p);
    ctxs |= 1u << (parts[p]->ctx & 31);
    xcds |= 1u << (parts[p]->xcd & 31);
  }
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    return std::make_tuple(parts[a]->ctx, parts[a]->gpu, parts[a]->xcd) <
           std::make_tuple(parts[b]->ctx, parts[b]->gpu, parts[b]->xcd);
  });
  const size_t online = std::min(order.size(), t.slots.size());
  for (size_t k = 0; k < t.slots.size(); ++k) {
    Slot& v = *slots[t.slots[k]];
    if (k < online) {
      if (v.pause_flags & VPF_DOWN) {
        v.pause_flags &= ~VPF_DOWN;
        v.home = order[k];
        v.soft = m;
        v.class_home = v.home;
        if (!v.is_running) {
          v.processor = v.home;
          v.home = -1;
        }
        vcpu_wake(v);
      } else {
        place_class(v, m, order[k]);
      }
    } else if (!(v.pause_flags & VPF_DOWN)) {
      v.pause_flags |= VPF_DOWN;
      v.class_home = -1;
      v.soft = Mask();
      vcpu_sleep_nosync(v);
    }
  }
  t.budget_shared = false;
  t.budget_ctx = ctxs | ((xcds & 0xffu) << 8);
  emit(TRC_CLASS, 0, t.id, (uint32_t)t.cls, (uint32_t)m.weight());
}

void Engine::budget_layout(Pool& pl, int64_t n, bool force) {
  const int64_t present_ns = (int64_t)std::max(0, boot.present_us) * 1000;
  std::vector<std::pair<int, int>> sig;  // (id, class) of present tenants, id order
  for (auto& tp : tenants) {
    if (!tp || !tp->alive || !tp->priv || tp->pool != pl.id) continue;
    Tenant& t = *tp;
    bool busy = false;
    for (int sid : t.slots) {
      const Slot& v = *slots[sid];
      if (!(v.pause_flags & VPF_BLOCKED) && v.pause_count == 0) busy = true;
    }
    if (busy && t.pause_count == 0) t.last_busy = n;
    // class -1: busy but not classified yet
    const bool present = n - t.last_busy <= present_ns;
    if (present) {  // mem_split: light = busy at under ~half of the class ticks
      t.busy_ewma += ((busy ? 1.0 : 0.0) - t.busy_ewma) / 16.0;
      if (t.light ? t.busy_ewma > 0.6 : t.busy_ewma < 0.4) t.light = !t.light;
    }
    // probe_max_us: a tenant that is present but blocked at class ticks (a
    // latency tenant: 100 us requests every 2 ms) never fills a clean
    // counter window; after probe_max_us it is laid out as memory class.  A
    // backlogged tenant is never expired -- it only needs its first clean
    // window (expiring one laid a GEMM out on a single memory SE next to a
    // stream in the live phase test, and the two grids stalled each other)
    int cls = t.cls;
    if (cls >= 0) {
      t.unclassified_since = INT64_MIN / 2;
      t.probe_gaps = false;
    } else if (present && t.unclassified_since == INT64_MIN / 2) {
      t.unclassified_since = n;  // (an absence does not restart the probe clock)
    } else if (present) {
      if (!busy) t.probe_gaps = true;
      if (t.probe_gaps && boot.probe_max_us > 0 && n - t.unclassified_since > (int64_t)boot.probe_max_us * 1000) {
        cls = 1;
        perfc.incr(PC_probe_expired);
      }
    }
    if (present) sig.emplace_back(t.id, cls);
    else t.budget_ctx = 0;
  }
  // class_pin_us: a flapping compute-phase tenant joins the memory region
  // when that region is time-shared already (two or more other memory-class
  // tenants): a fourth co-sharer costs each of them a quarter of their turns,
  // while its moves into the compute region halved the GEMM tenant's SEs for
  // no gain of its own (phase-ts).  Next to a single memory tenant it would
  // halve that tenant's SEs instead (phase mix: measured -0.008), so there it
  // keeps moving.
  {
    const int64_t pin_ns = (int64_t)std::max(0, boot.class_pin_us) * 1000;
    int mem = 0;
    for (auto& e : sig) mem += e.second == 1;
    for (auto& e : sig) {
      Tenant& t = *tenants[e.first];
      if (e.second == 0 && mem >= 2 && t.flapping(n, pin_ns)) e.second = 1;
      t.lay_cls = e.second;
    }
  }
  std::vector<int> light;
  if (boot.mem_split)
    for (auto& e : sig)
      if (tenants[e.first]->light) light.push_back(e.first);
  if (!force && sig == pl.budget_sig && light == pl.budget_light) return;
  pl.budget_sig = sig;
  pl.budget_light = light;
  perfc.incr(PC_relayout);
  // Probe layout: while a present tenant is not classified yet, every
  // present tenant gets an exclusive, equal share of the pool's partitions
  // (dealt round-robin in context-major order, so each share spans SEs and
  // XCDs).  Exclusive ownership is what makes a tenant's counters
  // attributable -- a tenant time-sharing partitions never gets a clean
  // window, so it would never be classified -- and a share per tenant keeps
  // the warm-up fair.  The class layout follows once every tenant has a class.
  bool probe = false;
  for (auto& e : sig) probe |= e.second < 0;
  int nctx = 0;
  uint32_t xall = 0;
  for (int p = pl.cpus.first(); p >= 0; p = pl.cpus.next(p + 1)) {
    nctx = std::max(nctx, parts[p]->ctx + 1);
    xall |= 1u << (parts[p]->xcd & 31);
  }
  if (nctx <= 0) return;
  const int nx = __builtin_popcount(xall);
  uint32_t ctx_all = 0;
  for (int x = 0; x < nctx; ++x) ctx_all |= 1u << x;
  // XCD blocks: tenant i of k gets nx/k whole XCDs (the first nx%k one more).
  auto xcd_block = [&](int i, int k) {
    int at = 0;
    for (int j = 0; j < i; ++j) at += nx / k + (j < nx % k ? 1 : 0);
    const int sz = nx / k + (i < nx % k ? 1 : 0);
    uint32_t m = 0;
    int seen = 0;
    for (int x = 0; x < 32; ++x)
      if ((xall >> x) & 1) {
        if (seen >= at && seen < at + sz) m |= 1u << x;
        ++seen;
      }
    return m;
  };
  // Two present tenants in SE-exclusive mode: the probe shares are the two
  // class halves (a classified tenant keeps its class's half, an unclassified
  // one takes the other).  A torch tenant on the shim launches a whole slice
  // on a queue masked to its half only when it owns a clean half of every
  // XCD; with XCD blocks both tenants' slices ran unmasked over each other
  // until the newcomer was classified (config #5: ~1 s of 15-20 ms decode
  // steps whenever the trainer arrived, profiles/r4/llm5_s25.txt).
  const int psplit = std::max(1, boot.class_split);
  if (probe && sig.size() == 2 && psplit > 1 && psplit < nctx) {
    const uint32_t lo = (1u << psplit) - 1, hi = ctx_all & ~lo;
    int first = 0;  // the tenant that takes the compute half (contexts [0, split))
    if (sig[0].second == 1 || sig[1].second == 0) first = 1;
    // Equal halves are the same hardware: two tenants that already hold one
    // half each stay where they are, and the pool's orientation (mirror)
    // follows the classified one -- config #5's trainer, classified while the
    // decode tenant is still probing, used to swap halves with it (both
    // tenants' CU masks, ~1 s of slow steps; profiles/r6/s35_llm5.json).
    if (2 * psplit == nctx) {
      auto half_of = [&](const Tenant& t) {
        const uint32_t b = t.budget_ctx & 0xFFu;
        return !b ? -1 : (b & ~lo) == 0 ? 0 : (b & ~hi) == 0 ? 1 : -1;
      };
      const int h0 = half_of(*tenants[sig[0].first]), h1 = half_of(*tenants[sig[1].first]);
      if (h0 >= 0 && h1 >= 0 && h0 != h1) {
        first = h0 == 0 ? 0 : 1;  // the tenant on the lower half keeps it
        for (int i = 0; i < 2; ++i)
          if (sig[i].second >= 0) {
            const bool m = (sig[i].second == 0) != ((i == first) ? true : false);
            if (m != pl.mirror) perfc.incr(PC_mirror);
            pl.mirror = m;
          }
      }
    }
    for (int i = 0; i < 2; ++i) {
      Tenant& t = *tenants[sig[i].first];
      t.budget_shared = false;
      place_budget(t, pl, i == first ? lo : hi, 0, 0);
    }
    perfc.incr(PC_probe_layout);
    process_softirqs();
    return;
  }
  if (probe && (int)sig.size() <= nx) {
    for (size_t i = 0; i < sig.size(); ++i) {
      Tenant& t = *tenants[sig[i].first];
      t.budget_shared = false;
      place_budget(t, pl, ctx_all, 0, xcd_block((int)i, (int)sig.size()));
    }
    perfc.incr(PC_probe_layout);
    process_softirqs();
    return;
  }
  if (probe) {  // more tenants than XCDs: deal single partitions
    std::vector<int> order;
    for (int p = pl.cpus.first(); p >= 0; p = pl.cpus.next(p + 1)) order.push_back(p);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
      return std::make_tuple(parts[a]->ctx, parts[a]->gpu, parts[a]->xcd) <
             std::make_tuple(parts[b]->ctx, parts[b]->gpu, parts[b]->xcd);
    });
    const size_t k = sig.size();
    for (size_t i = 0; i < k; ++i) {
      Tenant& t = *tenants[sig[i].first];
      Mask m;
      std::vector<int> homes;
      for (size_t j = i; j < order.size(); j += k) {
        m.set(order[j]);
        homes.push_back(order[j]);
      }
      if (homes.empty()) {  // more tenants than partitions: share one
        m.set(order[i % order.size()]);
        homes.push_back(order[i % order.size()]);
      }
      for (size_t s = 0; s < t.slots.size(); ++s) {
        Slot& v = *slots[t.slots[s]];
        if (s < homes.size()) {
          if (v.pause_flags & VPF_DOWN) {
            v.pause_flags &= ~VPF_DOWN;
            v.soft = m;
            v.class_home = homes[s];
            if (!v.is_running) v.processor = homes[s];
            vcpu_wake(v);
          } else {
            place_class(v, m, homes[s]);
          }
        } else if (!(v.pause_flags & VPF_DOWN)) {
          v.pause_flags |= VPF_DOWN;
          v.class_home = -1;
          v.soft = Mask();
          vcpu_sleep_nosync(v);
        }
      }
      t.budget_ctx = 0;
      t.budget_shared = false;
    }
    perfc.incr(PC_probe_layout);
    process_softirqs();
    return;
  }
  const int split = std::min(std::max(1, boot.class_split), nctx);
  std::vector<int> cls_t[2];
  for (auto& e : sig) cls_t[e.second & 1].push_back(e.first);
  // The two class halves are the same hardware when they are equal (SEs
  // {0,1} and {2,3} of every XCD): which class holds which half only decides
  // how many tenants move.  Keep the orientation that leaves more tenants on
  // the half they hold -- a classifier that swaps two tenants' classes
  // (config #5: the trainer's optimizer step streams 16 GB and out-misses the
  // fp8 decode over some windows) then costs no relayout at all, instead of
  // swapping both tenants' CU masks back and forth (profiles/r6/s28: decode
  // ~45 % of its slices on the other half, aggregate 1.19 against 1.24
  // without the swaps).
  if (!cls_t[0].empty() && !cls_t[1].empty() && 2 * split == nctx) {
    const uint32_t lo_m = (1u << split) - 1, hi_m = ((1u << nctx) - 1) & ~lo_m;
    int nat = 0, mir = 0;
    for (int c = 0; c < 2; ++c)
      for (int id : cls_t[c]) {
        const uint32_t b = tenants[id]->budget_ctx & 0xFFu;
        const int h = !b ? -1 : (b & ~lo_m) == 0 ? 0 : (b & ~hi_m) == 0 ? 1 : -1;
        if (h >= 0) (h == c ? nat : mir)++;
      }
    if (mir != nat) {
      const bool m = mir > nat;
      if (m != pl.mirror) perfc.incr(PC_mirror);
      pl.mirror = m;
    }
  } else {
    pl.mirror = false;
  }
  for (int c = 0; c < 2; ++c) {
    if (cls_t[c].empty()) continue;
    int lo = 0, hi = nctx;  // class region [lo, hi)
    if (!cls_t[0].empty() && !cls_t[1].empty()) {
      if ((c == 0) != pl.mirror) hi = split;
      else lo = split;
    }
    const int r = hi - lo, k = (int)cls_t[c].size();
    if (k > r && boot.class_budget >= 2 && k <= nx) {
      // Crowded region, spatial split: each tenant gets the region's SEs of
      // a block of whole XCDs (its own L2s: the per-XCD L2 misses become
      // exactly attributable too) -- the static split a human would pick,
      // re-derived whenever the classes or the present tenants change.
      uint32_t reg = 0;
      for (int x = lo; x < hi; ++x) reg |= 1u << x;
      for (int i = 0; i < k; ++i) {
        Tenant& t = *tenants[cls_t[c][i]];
        t.budget_shared = false;
        place_budget(t, pl, reg, 0, xcd_block(i, k));
      }
      continue;
    }
    if (k > r && c == 1 && boot.mem_split) {
      // Crowded memory region, split by partitions (boot mem_split): the
      // region's partitions in context-major order, an equal contiguous block
      // per backlogged tenant (a block of 4 of 16 is one SE of 4 XCDs), and a
      // small one -- an eighth of the region -- per light tenant, at the end.
      // Measured on the slo mix (profiles/r6/s20): a hand layout of this shape
      // 1.344 against 1.267 time-shared -- the MALL-sized tenant keeps 0.38 of
      // its solo rate on 48 CUs and 0.23 on a third of the whole region's time.
      std::vector<int> reg;
      for (int p = pl.cpus.first(); p >= 0; p = pl.cpus.next(p + 1))
        if (parts[p]->ctx >= lo && parts[p]->ctx < hi) reg.push_back(p);
      std::stable_sort(reg.begin(), reg.end(), [&](int a, int b) {
        return std::make_tuple(parts[a]->ctx, parts[a]->gpu, parts[a]->xcd) <
               std::make_tuple(parts[b]->ctx, parts[b]->gpu, parts[b]->xcd);
      });
      std::vector<int> heavy, lite;
      for (int id : cls_t[c]) (tenants[id]->light ? lite : heavy).push_back(id);
      if (heavy.empty()) heavy.swap(lite);
      const int P = (int)reg.size();
      int lp = lite.empty() ? 0 : std::max(1, P / 8);
      while (!lite.empty() && lp > 1 && (int)lite.size() * lp > P / 2) --lp;
      // mem_split 2: the light tenants' blocks overlap the last backlogged
      // tenant's instead of sitting idle between requests -- a request
      // BOOST-preempts that tenant on them
      const bool overlap = boot.mem_split >= 2;
      const int hp = overlap ? P : P - (int)lite.size() * lp, nh = (int)heavy.size();
      if (nh > 0 && hp >= nh) {
        int at = 0;
        auto give = [&](int id, int sz) {
          Mask m;
          for (int j = at; j < at + sz && j < P; ++j) m.set(reg[j]);
          at += sz;
          place_parts(*tenants[id], pl, m);
        };
        // Which backlogged tenant gets which block: greedily the pair with
        // the most partitions the tenant holds already (its online slots'
        // homes), so a tenant joining or leaving the region (a phase change)
        // moves as few partitions as it can -- each moved partition is a
        // revocation of the tenant that held it.  Newcomers take what is left.
        std::vector<int> bstart(nh), bsize(nh), owner(nh, -1);
        for (int i = 0, a = 0; i < nh; ++i) {
          bstart[i] = a;
          bsize[i] = hp / nh + (i < hp % nh ? 1 : 0);
          a += bsize[i];
        }
        std::vector<std::vector<int>> ov(nh, std::vector<int>(nh, 0));
        for (int ti = 0; ti < nh; ++ti)
          for (int sid : tenants[heavy[ti]]->slots) {
            const Slot& v = *slots[sid];
            if (v.class_home < 0 || (v.pause_flags & VPF_DOWN)) continue;
            for (int bi = 0; bi < nh; ++bi)
              for (int j = bstart[bi]; j < bstart[bi] + bsize[bi]; ++j)
                if (reg[j] == v.class_home) ov[ti][bi]++;
          }
        std::vector<bool> tdone(nh, false);
        for (int round = 0; round < nh; ++round) {
          int bt = -1, bb = -1, best = 0;
          for (int ti = 0; ti < nh; ++ti)
            for (int bi = 0; bi < nh && !tdone[ti]; ++bi)
              if (owner[bi] < 0 && ov[ti][bi] > best) best = ov[ti][bi], bt = ti, bb = bi;
          if (bt < 0) break;
          owner[bb] = bt;
          tdone[bt] = true;
        }
        for (int bi = 0, ti = 0; bi < nh; ++bi)
          if (owner[bi] < 0) {
            while (tdone[ti]) ++ti;
            owner[bi] = ti;
            tdone[ti] = true;
          }
        for (int bi = 0; bi < nh; ++bi) {
          at = bstart[bi];
          give(heavy[owner[bi]], bsize[bi]);
        }
        // mem_split 2: the light blocks sit at the end of the LARGEST
        // backlogged block (the first: it took the remainder), so the
        // tenant that BOOSTed requests preempt is the one with a partition
        // to spare (slo: the two streams kept 0.32 / 0.22 of their solo
        // rates with the light block on the smaller one's)
        at = overlap ? std::max(0, bstart[0] + bsize[0] - (int)lite.size() * lp) : hp;
        for (int id : lite) give(id, lp);
        perfc.incr(PC_mem_split);
        continue;
      }
    }
    if (k > r) {  // time-shared region: every tenant on all of it, staggered by whole contexts
      uint32_t all = 0;
      for (int x = lo; x < hi; ++x) all |= 1u << x;
      int per = 0;
      for (int p = pl.cpus.first(); p >= 0; p = pl.cpus.next(p + 1)) per += parts[p]->ctx == lo;
      for (int i = 0; i < k; ++i) {
        Tenant& t = *tenants[cls_t[c][i]];
        t.budget_shared = true;
        place_budget(t, pl, all, (i % r) * per);
      }
      continue;
    }
    // aligned blocks: sizes r/k, the first r%k tenants one more; with r = 4
    // and k = 3 that is 2+1+1 (a 2-block always starts on an even context)
    int at = lo;
    for (int i = 0; i < k; ++i) {
      const int sz = r / k + (i < r % k ? 1 : 0);
      uint32_t msk = 0;
      for (int x = at; x < at + sz; ++x) msk |= 1u << x;
      at += sz;
      Tenant& t = *tenants[cls_t[c][i]];
      t.budget_shared = false;
      place_budget(t, pl, msk, 0);
    }
  }
  process_softirqs();
}

void Engine::classify_tick(int64_t n) {
  std::vector<int> changed;
  for (auto& tp : tenants) {
    if (!tp || !tp->alive || !tp->priv) continue;
    Tenant& t = *tp;
    Pool* pl = pool(t.pool);
    if (!pl) continue;
    const int c = pl->sched->classify(t);
    if (c < 0) continue;
    if (c != t.cls_pending) {
      t.cls_pending = c;
      t.cls_count = 1;
    } else {
      t.cls_count++;
    }
    if (t.cls_count < std::max(1, boot.class_dwell) || c == t.cls) {
      // Stolen across classes and no longer running: back to its class home.
      // Stacked on an XCD that hosts more of the tenant's slots than its home
      // XCD does (an in-class steal of a slot that waited behind a sibling):
      // home too, even while running -- in a fully
      // busy pool nothing else would ever undo it, and the tenant would miss
      // XCDs it is entitled to.
      // A slot alone on a foreign XCD whose home XCD has none of the
      // tenant's slots goes home as well: neutral for the slot, but it
      // unblocks a chain of displaced slots (B stacked behind A's home...).
      auto on_xcd = [&](int part, size_t skip) {
        int n = 0;
        for (size_t j = 0; j < t.slots.size(); ++j) {
          const Slot& w = *slots[t.slots[j]];
          if (j == skip || !runnable(w)) continue;
          const Partition& Q = *parts[w.processor];
          n += Q.gpu == parts[part]->gpu && Q.xcd == parts[part]->xcd;
        }
        return n;
      };
      uint32_t home_ctx = 0;  // contexts (shader engines) the tenant's class homes use
      for (int sid : t.slots)
        if (slots[sid]->class_home >= 0) home_ctx |= 1u << (parts[slots[sid]->class_home]->ctx & 31);
      for (size_t k = 0; k < t.slots.size(); ++k) {
        Slot& v = *slots[t.slots[k]];
        if (!runnable(v) || v.class_home < 0 || v.processor == v.class_home) continue;
        if (boot.class_budget && boot.class_split > 1) {
          // Budget layout: every online slot has a partition of its own, so
          // a slot away from home (stolen while its tenant's share was
          // idle, or displaced by a relayout onto a sibling's home) always
          // goes back; a chain of displaced slots unwinds in a few ticks.
          send_home(v);
          continue;
        }
        const Partition& P = *parts[v.processor];
        const Partition& H = *parts[v.class_home];
        const bool stray = !v.is_running && !v.soft.empty() && !v.soft.test(v.processor);
        const int here = on_xcd(v.processor, k), there = on_xcd(v.class_home, k);
        const bool foreign = P.gpu != H.gpu || P.xcd != H.xcd;
        // SE-exclusive mode: a slot on a shader engine outside its tenant's
        // home SEs is misplaced even when its XCD holds the right number of
        // the tenant's slots -- the runner's CU-masked stream covers one
        // class half ({0,1} or {2,3}), so a tenant holding SEs {0,3}
        // launches unmasked and its workgroups queue behind the other
        // owner's SEs (config #2 measured 0.73 vs 1.26 under none).  It goes
        // to a home partition none of its siblings occupies, preferably on
        // its own XCD, trading homes with the sibling that partition was
        // home to (homes stay one per partition).
        auto occupied = [&](int part) {
          for (size_t j = 0; j < t.slots.size(); ++j)
            if (j != k && runnable(*slots[t.slots[j]]) && slots[t.slots[j]]->processor == part) return true;
          return false;
        };
        // Stacked behind a sibling on one partition while its own home --
        // free of siblings -- sits on the same XCD: in a fully busy pool no
        // steal ever separates them, and with the class's SEs time-shared
        // (more slots than partitions) the tenant then holds one SE of that
        // XCD permanently while the gang alternates everywhere else.
        const bool stacked = !foreign && occupied(v.processor) && !occupied(v.class_home);
        bool wrong_se = false;
        if (boot.class_split > 1 && !((home_ctx >> P.ctx) & 1)) {
          int target = -1;
          size_t owner = k;
          for (size_t j = 0; j < t.slots.size(); ++j) {
            const int hp = slots[t.slots[j]]->class_home;
            if (hp < 0 || occupied(hp)) continue;
            const bool local = parts[hp]->gpu == P.gpu && parts[hp]->xcd == P.xcd;
            if (target < 0 || (local && !(parts[target]->gpu == P.gpu && parts[target]->xcd == P.xcd))) {
              target = hp;
              owner = j;
            }
          }
          if (target >= 0) {
            if (owner != k) std::swap(slots[t.slots[owner]]->class_home, v.class_home);
            wrong_se = true;
          }
        }
        if (stray || wrong_se || stacked || (foreign && (there < here || (there == 0 && here == 0)))) send_home(v);
      }
      continue;
    }
    pl->sched->class_changed(t, t.cls, c);
    if (t.cls >= 0) {  // a change of class (not the first classification)
      t.cls_chg_ns[0] = t.cls_chg_ns[1];
      t.cls_chg_ns[1] = t.cls_chg_ns[2];
      t.cls_chg_ns[2] = n;
    }
    t.cls = c;
    perfc.incr(PC_class_change);
    changed.push_back(t.id);
  }
  // Class layout per pool: the classes present among its classified
  // tenants.  With both present, compute owns contexts [0, class_split) and
  // memory the rest; with one class only, that class spans every context (two
  // GEMM tenants each take two SEs of every XCD instead of time-sharing two
  // while the memory SEs idle -- config #2).  A layout change re-places every
  // classified tenant of the pool; otherwise only the re-classified ones.
  for (auto& pp : pools) {
    if (!pp) continue;
    Pool& pl = *pp;
    if (boot.class_split > 1 && boot.class_budget) {
      bool any_changed = false;
      for (auto& tp : tenants)
        if (tp && tp->alive && tp->pool == pl.id &&
            std::find(changed.begin(), changed.end(), tp->id) != changed.end())
          any_changed = true;
      budget_layout(pl, n, any_changed);
      continue;
    }
    int layout = 0;
    for (auto& tp : tenants)
      if (tp && tp->alive && tp->priv && tp->pool == pl.id && tp->cls >= 0) layout |= 1 << tp->cls;
    const bool relayout = layout != pl.class_layout;
    pl.class_layout = layout;
    for (auto& tp : tenants) {
      if (!tp || !tp->alive || !tp->priv || tp->pool != pl.id || tp->cls < 0) continue;
      if (relayout || std::find(changed.begin(), changed.end(), tp->id) != changed.end())
        place_tenant_class(*tp, pl, layout);
    }
  }
  process_softirqs();
  timer_set(class_timer_, n + (int64_t)std::max(100, boot.class_period_us) * 1000);
}

// ------------------------------------------------------------ heartbeats ---

void Engine::heartbeat_check(int64_t n) {
  const int64_t tmo = (int64_t)boot.heartbeat_timeout_us * 1000;
  for (auto& t : tenants) {
    if (!t || !t->alive || t->id == 0) continue;
    if (n - t->last_heartbeat > tmo && t->pause_count == 0) {
      // Reclaim: the tenant is declared dead; its partitions go to others.
      t->pause_count++;
      for (int sid : t->slots) vcpu_sleep_nosync(*slots[sid]);
      perfc.incr(PC_tenant_dead);
      emit(TRC_DEAD, 0, t->id);
      printk(fmt("(GPBS) tenant %d (%s) missed heartbeats for %" PRId64 "us: paused\n", t->id, t->name.c_str(),
                 (n - t->last_heartbeat) / 1000));
    }
  }
  timer_set(hb_timer_, n + tmo / 2);
}

// -------------------------------------------------------------- watchdogs ---
// SCHEDOP_watchdog (X:xen/common/schedule.c:738-788): a tenant arms up to
// GPBS_WATCHDOGS timers and must re-arm them before they expire; an expired
// one shuts the tenant down (domain_shutdown(d, SHUTDOWN_watchdog) there; here
// its slots are paused and its partitions go to the other tenants).  Unlike
// the heartbeat detector, the deadline is the tenant's own choice.

int Engine::watchdog(int tid, uint32_t id, uint32_t timeout_ms) {
  Tenant* t = tenant(tid);
  if (!t || !t->alive) return GPBS_ENOENT;
  if (id > (uint32_t)GPBS_WATCHDOGS) return GPBS_EINVAL;
  if (id == 0) {
    for (int k = 0; k < GPBS_WATCHDOGS; ++k) {
      if (t->wd_inuse & (1u << k)) continue;
      t->wd_inuse |= 1u << k;
      if (t->wd_timer[k] < 0) t->wd_timer[k] = timer_init([this, tid, k](int64_t) { watchdog_fire(tid, k); });
      timer_set(t->wd_timer[k], now() + (int64_t)timeout_ms * 1000000);
      return k + 1;
    }
    return GPBS_ENOSPC;
  }
  const int k = (int)id - 1;
  if (!(t->wd_inuse & (1u << k))) return GPBS_EINVAL;
  if (timeout_ms == 0) {
    timer_stop(t->wd_timer[k]);
    t->wd_inuse &= ~(1u << k);
  } else {
    timer_set(t->wd_timer[k], now() + (int64_t)timeout_ms * 1000000);
  }
  return GPBS_OK;
}

void Engine::watchdog_fire(int tid, int k) {
  Tenant* t = tenant(tid);
  if (!t || !t->alive || t->shutdown) return;  // is_shutting_down / is_dying
  printk(fmt("(GPBS) Watchdog timer %d fired for tenant %d (%s)\n", k + 1, t->id, t->name.c_str()));
  t->shutdown = GPBS_SHUTDOWN_WATCHDOG;
  t->pause_count++;
  for (int sid : t->slots) vcpu_sleep_nosync(*slots[sid]);
  perfc.incr(PC_watchdog_fired);
  emit(TRC_DEAD, 0, t->id, GPBS_SHUTDOWN_WATCHDOG);
  process_softirqs();
}

void Engine::watchdog_kill(Tenant& t) {
  for (int k = 0; k < GPBS_WATCHDOGS; ++k)
    if (t.wd_timer[k] >= 0) {
      timer_kill(t.wd_timer[k]);
      t.wd_timer[k] = -1;
    }
  t.wd_inuse = 0;
}

// --------------------------------------------------------- observability ---

void Engine::printk(const std::string& s) {
  console_ += s;
  if (console_.size() > (1u << 20)) console_.erase(0, console_.size() - (1u << 19));
}

std::string Engine::dmesg(bool clear) {
  std::string s = console_;
  if (clear) console_.clear();
  return s;
}

std::string Engine::dump_runq() {
  std::string o;
  o += fmt("sched_smt_power_savings: %s\n", boot.smt_power_savings ? "enabled" : "disabled");
  o += fmt("NOW=0x%016" PRIx64 "\n", (uint64_t)now());
  std::string free_cpus;
  for (auto& p : parts)
    if (p->pool < 0) free_cpus += fmt("%d ", p->id);
  o += "Idle cpupool:\n";
  o += "  free partitions: " + (free_cpus.empty() ? std::string("none") : free_cpus) + "\n";
  for (auto& pl : pools) {
    if (!pl) continue;
    o += fmt("Cpupool %d:\n", pl->id);
    o += fmt("Scheduler: %s (%s)\n", pl->sched->name(), pl->sched->opt_name());
    pl->sched->dump_settings(o);
    for (int c = pl->cpus.first(); c >= 0; c = pl->cpus.next(c + 1)) {
      o += fmt("CPU[%02d] (gpu%d xcd%d.%d) ", c, parts[c]->gpu, parts[c]->xcd, parts[c]->ctx);
      pl->sched->dump_cpu_state(c, o);
    }
  }
  return o;
}

std::string Engine::dump_domains() {
  std::string o = fmt("'q' pressed -> dumping domain info (now=0x%016" PRIx64 ")\n", (uint64_t)now());
  for (auto& t : tenants) {
    if (!t || !t->alive) continue;
    o += fmt("General information for domain %d (%s):\n", t->id, t->name.c_str());
    o += fmt("    pause_count=%d pool=%d pending_requests=%" PRIu64 "\n", t->pause_count, t->pool,
             t->pending_requests);
    o += fmt("VCPU information and callbacks for domain %d:\n", t->id);
    for (int sid : t->slots) {
      Slot& v = *slots[sid];
      o += fmt("    VCPU%d: CPU%d [has=%c] cpu_affinity=%s\n", v.index, v.processor, v.is_running ? 'T' : 'F',
               v.affinity.weight() >= kMaxPartitions ? "all" : v.affinity.str().c_str());
      o += fmt("    pause_count=%d pause_flags=%x\n", v.pause_count, v.pause_flags);
      // keyhandler.c:294 pmuinfo line
      o += fmt("pmuinfo: pmc[0]=%" PRIu64 "    pmc[1]=%" PRIu64 "    pmc[2]=%" PRIu64 "    pmc[3]=%" PRIu64 "\n",
               v.pmc[0], v.pmc[1], v.pmc[2], v.pmc[3]);
    }
  }
  return o;
}

std::string Engine::dump_customized() {
  std::string o;
  for (auto& pl : pools) {
    if (!pl) continue;
    o += fmt("Cpupool %d:\n", pl->id);
    o += fmt("Scheduler: %s (%s)\n", pl->sched->name(), pl->sched->opt_name());
    pl->sched->dump_admin_conf(o);
  }
  return o;
}

std::string Engine::check_invariants() {
  std::string err;
  for (auto& pl : pools)
    if (pl) err += pl->sched->check();
  for (auto& p : parts) {
    Slot* c = slot(p->curr);
    if (!c) {
      err += fmt("cpu%d: curr slot missing\n", p->id);
      continue;
    }
    if (!c->is_running) err += fmt("cpu%d: curr slot %d not marked running\n", p->id, c->id);
    if (!c->is_idle() && c->processor != p->id) err += fmt("cpu%d: curr slot %d on cpu%d\n", p->id, c->id, c->processor);
  }
  for (auto& s : slots) {
    if (!s || s->is_idle() || !s->is_running) continue;
    if (parts[s->processor]->curr != s->id) err += fmt("slot %d running but not curr of cpu%d\n", s->id, s->processor);
  }
  return err;
}

std::string Engine::debug_keys(const std::string& keys) {
  std::string o;
  for (char k : keys) {
    std::string part;
    switch (k) {
      case 'r':
        part = dump_runq();
        break;
      case 'q':
        part = dump_domains();
        break;
      case 'z':
        part = dump_customized();
        break;
      case 'p': {  // perfc printall
        for (int i = 0; i < PC_COUNT; ++i) part += fmt("%-28s %" PRIu64 "\n", kPerfcNames[i], perfc.get((PerfcId)i));
        break;
      }
      case 'P':
        perfc.reset();
        part = "perfc reset\n";
        break;
      case 'c': {
        part = check_invariants();
        if (part.empty()) part = "invariants ok\n";
        break;
      }
      case 'h':
        part =
            " 'r' dump run queues\n 'q' dump domain (tenant) info\n 'z' dump customized settings (PBS)\n"
            " 'p' print performance counters\n 'P' reset performance counters\n 'c' check invariants\n";
        break;
      default:
        part = fmt("'%c' unknown key\n", k);
    }
    printk(part);
    o += part;
  }
  return o;
}

// ------------------------------------------------------ dispatcher thread --

int Engine::start() {
  if (boot.sim_clock) return GPBS_EINVAL;
  ApiLock g(this);
  if (running_) return GPBS_OK;
  running_ = true;
  thread_ = std::thread([this] { loop(); });
  return GPBS_OK;
}

int Engine::stop() {
  {
    ApiLock g(this);  // counted as a waiter: a dispatcher behind schedule hands off
    if (!running_) return GPBS_OK;
    running_ = false;
  }
  cv_.notify_all();
  if (thread_.joinable()) thread_.join();
  return GPBS_OK;
}

void Engine::kick() {
  kicked_ = true;
  cv_.notify_all();
}

void Engine::loop() {
  prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);  // µs-accurate quanta
  std::unique_lock<std::recursive_mutex> lk(mu);
  uint64_t t_acq = 0;
  auto held = [&](bool blocked, uint64_t wait_ns) {
    lock_depth_++;
    lockprof.acquired(blocked, wait_ns);
    t_acq = LockProfile::clock_ns();
  };
  auto releasing = [&] {
    lockprof.released(LockProfile::clock_ns() - t_acq);
    lock_depth_--;
  };
  auto relock = [&] {
    const uint64_t t0 = LockProfile::clock_ns();
    const bool blocked = !lk.try_lock();
    if (blocked) lk.lock();
    held(blocked, LockProfile::clock_ns() - t0);
  };
  held(false, 0);
  while (running_) {
    int64_t n = now();
    run_due(n);
    int64_t dl = next_deadline();
    kicked_ = false;
    n = now();
    if (dl <= n) {
      // Behind schedule: let blocked API callers in before catching up.
      if (api_waiters_.load(std::memory_order_relaxed) > 0) {
        lockprof.handoffs.fetch_add(1, std::memory_order_relaxed);
        releasing();
        lk.unlock();
        const int64_t until = mono_ns() + 200000;
        while (api_waiters_.load(std::memory_order_relaxed) > 0 && mono_ns() < until) std::this_thread::yield();
        relock();
      }
      continue;
    }
    int64_t wait = dl == INT64_MAX ? 50000000 : dl - n;
    if (wait > 40000) {
      releasing();
      cv_.wait_for(lk, std::chrono::nanoseconds(wait - 20000), [this] { return kicked_ || !running_; });
      held(false, 0);
    } else {
      // Final approach: drop the lock and spin-yield so API callers get in.
      releasing();
      lk.unlock();
      while (mono_ns() < dl && !kicked_) std::this_thread::yield();
      relock();
    }
  }
  releasing();
}

}  // namespace gpbs
