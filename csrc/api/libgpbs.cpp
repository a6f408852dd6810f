// libgpbs: the C ABI (libxl/libxc analog).  Validation mirrors libxl
// (X:tools/libxl/libxl.c:4007-4116) so every frontend (ctypes, RPC daemon,
// gpbsctl) sees the same ranges and error codes.
#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>

#include "../core/engine.h"
#include "../include/gpbs/gpbs.h"

using namespace gpbs;

struct gpbs_engine {
  Engine* e;
};

namespace gpbs {
const char* const kPerfcNames[PC_COUNT] = {
#define GPBS_PERFC_NAME(n) #n,
    GPBS_PERFC_LIST(GPBS_PERFC_NAME)
#undef GPBS_PERFC_NAME
};
}  // namespace gpbs

static_assert(sizeof(gpbs_adapt_state_t) == sizeof(AdaptState), "adapt state layout");
static_assert(sizeof(gpbs_adapt_params_t) == sizeof(AdaptParams), "adapt params layout");
static_assert(sizeof(gpbs_atc_params_t) == sizeof(AtcParams), "atc params layout");
static_assert(sizeof(gpbs_trace_record_t) == sizeof(TraceRecord), "trace layout");

#define LOCK(E) Engine::ApiLock _g((E)->e)
#define DONE(E)                 \
  do {                          \
    (E)->e->process_softirqs(); \
    (E)->e->flush_actuation();  \
    (E)->e->kick();             \
  } while (0)

static int copy_str(const std::string& s, char* out, int len) {
  if (!out || len <= 0) return (int)s.size();
  int n = (int)std::min<size_t>(s.size(), (size_t)len - 1);
  std::memcpy(out, s.data(), n);
  out[n] = 0;
  return (int)s.size();
}

static Tenant* live(gpbs_engine_t* e, int t) {
  Tenant* d = e->e->tenant(t);
  return d && d->alive ? d : nullptr;
}

int gpbs_tenant_pause(gpbs_engine_t* e, int t) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  d->pause_count++;
  for (int sid : d->slots) e->e->vcpu_sleep_nosync(*e->e->slots[sid]);
  DONE(e);
  return GPBS_OK;
}

int gpbs_tenant_unpause(gpbs_engine_t* e, int t) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  if (d->pause_count == 0) return GPBS_EINVAL;
  if (--d->pause_count == 0) {
    d->shutdown = 0;  // operator restart of a watchdog-shut-down tenant
    for (int sid : d->slots) e->e->vcpu_wake(*e->e->slots[sid]);
  }
  d->last_heartbeat = e->e->now();
  DONE(e);
  return GPBS_OK;
}

int gpbs_tenant_set_nslots(gpbs_engine_t* e, int t, int n) {
  LOCK(e);
  int r = e->e->tenant_set_nslots(t, n);
  DONE(e);
  return r;
}

int gpbs_slot_id(gpbs_engine_t* e, int t, int idx) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d || idx < 0 || idx >= (int)d->slots.size()) return GPBS_EINVAL;
  return d->slots[idx];
}

template <typename F>
static int each_slot(gpbs_engine_t* e, int t, int idx, F f) {
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  if (idx < 0) {
    for (int sid : d->slots) f(*e->e->slots[sid]);
  } else {
    if (idx >= (int)d->slots.size()) return GPBS_EINVAL;
    f(*e->e->slots[d->slots[idx]]);
  }
  return GPBS_OK;
}


extern "C" {

void gpbs_boot_defaults(gpbs_boot_params_t* p) {
  std::memset(p, 0, sizeof(*p));
  std::strncpy(p->sched, "credit", sizeof(p->sched) - 1);
  p->tslice_us = 100;        // CSCHED_DEFAULT_TSLICE_US (sched_credit.c:52)
  p->ratelimit_us = 1000;    // SCHED_DEFAULT_RATELIMIT_US (sched-if.h:21) -> clamped to tslice
  p->smt_power_savings = 0;
  p->tickle_one_idle = 1;
  p->default_yield = 0;
  p->migration_delay_us = 0;
  p->metric_period_us = 1000;  // CSCHED_METRIC_TICK_PERIOD
  p->slice_apply_us = 3000;    // CSCHED_TIME_APPLY
  p->sim_clock = 0;
  p->pmu_refresh_us = 1111;
  p->dom0_quirk = 1;
  p->heartbeat_timeout_us = 0;
  p->trace_capacity = 1 << 16;
  p->quantum_align_us = 0;
  p->coschedule = 0;
  p->class_period_us = 2000;
  p->boost_exclusive = 0;
  p->class_split = 0;
  p->idle_skip = 0;  // reference semantics (Appendix A feeds every period)
  p->class_dwell = 2;
  p->class_budget = 0;
  p->present_us = 10000;
  p->sibling_steal = 0;
  p->class_steal = 1;
  p->class_fall = 0;
  p->shared_q_us = 0;
  p->class_pin_us = 0;
  p->region_q = 0;
  p->switch_floor_x = 0;
  p->switch_floor_max_us = 0;
  p->region_vt = 0;
  p->slo_cap = 0;
  p->probe_max_us = 0;
  p->mem_split = 0;
  AdaptParams a;
  std::memcpy(&p->adapt, &a, sizeof(a));
  AtcParams t;
  std::memcpy(&p->atc, &t, sizeof(t));
}

int gpbs_abi_version(void) { return GPBS_ABI_VERSION; }

const char* gpbs_strerror(int err) {
  switch (err) {
    case GPBS_OK: return "ok";
    case GPBS_EINVAL: return "invalid argument";
    case GPBS_ENOENT: return "no such tenant/pool";
    case GPBS_EBUSY: return "busy";
    case GPBS_ENOMEM: return "out of memory";
    case GPBS_ERANGE: return "value out of range";
    case GPBS_ENOSPC: return "no space";
    case GPBS_EEXIST: return "already exists";
    default: return "unknown error";
  }
}

gpbs_engine_t* gpbs_engine_create(const gpbs_boot_params_t* p) {
  gpbs_boot_params_t d;
  if (!p) {
    gpbs_boot_defaults(&d);
    p = &d;
  }
  auto* h = new gpbs_engine;
  h->e = new Engine(*p);
  if (h->e->pools.empty() || !h->e->pools[0]) {
    delete h->e;
    delete h;
    return nullptr;
  }
  h->e->fault_parse(std::getenv("GPBS_FAULT"));
  return h;
}

int gpbs_fault_set(gpbs_engine_t* e, const char* spec) {
  LOCK(e);
  return e->e->fault_parse(spec);
}

int64_t gpbs_fault_fire(gpbs_engine_t* e, const char* kind) {
  static const char* names[Engine::F_NKIND] = {"counter_drop", "counter_reset", "heartbeat_drop", "actuate_delay",
                                               "timer_jitter", "rank_hang", "torn_page"};
  if (!e || !kind) return -1;
  LOCK(e);
  for (int k = 0; k < Engine::F_NKIND; ++k)
    if (std::strcmp(kind, names[k]) == 0) {
      if (!e->e->fault(k)) return -1;
      e->e->emit(TRC_FAULT, 0, (uint32_t)k, (uint32_t)e->e->fault_param[k]);
      return e->e->fault_param[k] > 0 ? e->e->fault_param[k] : 0;
    }
  return -1;
}

// A gang epoch missed its deadline on this rank: degrade to local scheduling
// (every cross-GPU gang window is cleared, so no tenant is favoured or
// excluded for the sake of peers that may never arrive).
int gpbs_gang_timeout(gpbs_engine_t* e, uint32_t epoch, uint32_t rank, uint32_t waited_us) {
  LOCK(e);
  Engine* E = e->e;
  for (auto& t : E->tenants)
    if (t && t->alive) {
      t->gang_state = 0;
      t->gang_until = 0;
    }
  for (auto& p : E->parts) E->raise_softirq(p->id);
  E->perfc.incr(PC_gang_timeout);
  E->emit(TRC_GANG_TIMEOUT, rank, epoch, rank, waited_us);
  char msg[160];
  std::snprintf(msg, sizeof(msg), "(GPBS) gang epoch %u: deadline missed after %u us on rank %u, scheduling locally\n",
                epoch, waited_us, rank);
  E->printk(msg);
  DONE(e);
  return GPBS_OK;
}

int gpbs_fault_hits(gpbs_engine_t* e, uint64_t* out, int n) {
  LOCK(e);
  const int k = std::min<int>(n, Engine::F_NKIND);
  for (int i = 0; i < k; ++i) out[i] = e->e->fault_hits[i];
  return k;
}

void gpbs_engine_destroy(gpbs_engine_t* e) {
  if (!e) return;
  delete e->e;
  delete e;
}

int gpbs_partition_add(gpbs_engine_t* e, int gpu, int xcd) {
  LOCK(e);
  return e->e->partition_add(gpu, xcd, 0);
}

int gpbs_partition_add_ctx(gpbs_engine_t* e, int gpu, int xcd, int ctx) {
  LOCK(e);
  return e->e->partition_add(gpu, xcd, ctx);
}

int gpbs_num_partitions(gpbs_engine_t* e) {
  LOCK(e);
  return (int)e->e->parts.size();
}

int gpbs_pool_create(gpbs_engine_t* e, const char* name, const char* sched) {
  LOCK(e);
  if (!name || !*name) return GPBS_EINVAL;
  int r = e->e->pool_create(name, sched ? sched : "");
  DONE(e);
  return r;
}

int gpbs_pool_destroy(gpbs_engine_t* e, int pool) {
  LOCK(e);
  return e->e->pool_destroy(pool);
}

int gpbs_pool_rename(gpbs_engine_t* e, int pool, const char* name) {
  LOCK(e);
  Pool* p = e->e->pool(pool);
  if (!p || !name || !*name) return GPBS_EINVAL;
  for (auto& q : e->e->pools)
    if (q && q->name == name && q.get() != p) return GPBS_EEXIST;
  p->name = name;
  return GPBS_OK;
}

int gpbs_pool_find(gpbs_engine_t* e, const char* name) {
  LOCK(e);
  for (auto& q : e->e->pools)
    if (q && name && q->name == name) return q->id;
  return GPBS_ENOENT;
}

int gpbs_pool_assign(gpbs_engine_t* e, int pool, int part) {
  LOCK(e);
  int r = e->e->pool_assign(pool, part);
  DONE(e);
  return r;
}

int gpbs_pool_unassign(gpbs_engine_t* e, int pool, int part) {
  LOCK(e);
  int r = e->e->pool_unassign(pool, part);
  DONE(e);
  return r;
}

int gpbs_pool_info(gpbs_engine_t* e, int pool, char* name, int name_len, char* sched, int sched_len, uint64_t* mask4,
                   int* n_tenants) {
  LOCK(e);
  Pool* p = e->e->pool(pool);
  if (!p) return GPBS_ENOENT;
  copy_str(p->name, name, name_len);
  copy_str(p->sched->opt_name(), sched, sched_len);
  if (mask4)
    for (int i = 0; i < 4; ++i) mask4[i] = p->cpus.w[i];
  if (n_tenants) {
    int n = 0;
    for (auto& t : e->e->tenants)
      if (t && t->alive && t->pool == pool) n++;
    *n_tenants = n;
  }
  return GPBS_OK;
}

int gpbs_pool_list(gpbs_engine_t* e, int* ids, int max) {
  LOCK(e);
  int n = 0;
  for (auto& p : e->e->pools)
    if (p) {
      if (ids && n < max) ids[n] = p->id;
      n++;
    }
  return n;
}

int gpbs_partition_info(gpbs_engine_t* e, int part, gpbs_partition_info_t* o) {
  LOCK(e);
  Engine& E = *e->e;
  if (part < 0 || part >= (int)E.parts.size()) return GPBS_EINVAL;
  Partition& P = *E.parts[part];
  std::memset(o, 0, sizeof(*o));
  o->id = P.id;
  o->gpu = P.gpu;
  o->xcd = P.xcd;
  o->ctx = P.ctx;
  o->pool = P.pool;
  Slot& c = *E.slots[P.curr];
  o->curr_slot = c.is_idle() ? -1 : c.id;
  o->curr_tenant = c.tenant;
  o->idle = c.is_idle();
  o->switches = P.switches;
  int rq = 0;
  for (auto& s : E.slots)
    if (s && !s->is_idle() && s->processor == part && !s->is_running && E.runnable(*s)) rq++;
  o->runq_len = rq;
  return GPBS_OK;
}

int gpbs_tenant_create(gpbs_engine_t* e, const char* name, int pool, int nslots, int weight, int cap) {
  LOCK(e);
  if (!name || !*name) return GPBS_EINVAL;
  int r = e->e->tenant_create(name, pool, nslots, weight, cap);
  DONE(e);
  return r;
}

int gpbs_tenant_destroy(gpbs_engine_t* e, int t) {
  LOCK(e);
  int r = e->e->tenant_destroy(t);
  DONE(e);
  return r;
}

int gpbs_tenant_find(gpbs_engine_t* e, const char* name) {
  LOCK(e);
  for (auto& t : e->e->tenants)
    if (t && t->alive && name && t->name == name) return t->id;
  return GPBS_ENOENT;
}

int gpbs_tenant_list(gpbs_engine_t* e, int* ids, int max) {
  LOCK(e);
  int n = 0;
  for (auto& t : e->e->tenants)
    if (t && t->alive) {
      if (ids && n < max) ids[n] = t->id;
      n++;
    }
  return n;
}

int gpbs_tenant_move(gpbs_engine_t* e, int t, int pool) {
  LOCK(e);
  int r = e->e->tenant_move(t, pool);
  DONE(e);
  return r;
}

int gpbs_slot_wake(gpbs_engine_t* e, int t, int idx) {
  LOCK(e);
  int r = each_slot(e, t, idx, [&](Slot& v) { e->e->vcpu_unblock(v); });
  DONE(e);
  return r;
}

int gpbs_slot_block(gpbs_engine_t* e, int t, int idx) {
  LOCK(e);
  int r = each_slot(e, t, idx, [&](Slot& v) { e->e->vcpu_block(v); });
  DONE(e);
  return r;
}

int gpbs_slot_yield(gpbs_engine_t* e, int t, int idx) {
  LOCK(e);
  int r = each_slot(e, t, idx, [&](Slot& v) {
    if (Scheduler* S = e->e->sched_of_tenant(v.tenant)) {
      S->yield(v);
      if (v.is_running) e->e->raise_softirq(v.processor);
    }
  });
  DONE(e);
  return r;
}

int gpbs_slot_pin(gpbs_engine_t* e, int t, int idx, const uint64_t* mask4) {
  LOCK(e);
  Mask m;
  for (int i = 0; i < 4; ++i) m.w[i] = mask4[i];
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  if ((m & e->e->pools[d->pool]->cpus).empty()) return GPBS_EINVAL;
  int r = each_slot(e, t, idx, [&](Slot& v) { e->e->set_affinity(v, m); });  // vcpu_set_affinity
  DONE(e);
  return r;
}

int gpbs_tenant_info(gpbs_engine_t* e, int t, gpbs_tenant_info_t* o) {
  LOCK(e);
  Engine& E = *e->e;
  Tenant* d = E.tenant(t);
  if (!d || !d->priv) return GPBS_ENOENT;
  std::memset(o, 0, sizeof(*o));
  o->id = d->id;
  o->pool = d->pool;
  o->nslots = (int)d->slots.size();
  o->paused = d->pause_count;
  o->alive = d->alive;
  o->shutdown = d->shutdown;
  copy_str(d->name, o->name, sizeof(o->name));
  if (Scheduler* S = E.sched_of_tenant(t)) S->fill_tenant_info(*d, *o);
  const int64_t n = E.now();
  for (int sid : d->slots) {
    Slot& v = *E.slots[sid];
    o->sched_count += v.sched_count;
    o->run_ns += v.rs_time[RS_RUNNING] + (v.rs == RS_RUNNING ? n - v.rs_entry : 0);
    o->online_slots += !(v.pause_flags & VPF_DOWN);
  }
  o->budget_ctx = d->budget_ctx;
  o->budget_shared = d->budget_shared;
  o->switch_cost_us = d->sw_cost_us;
  o->slo_us = d->slo_us;
  return GPBS_OK;
}

int gpbs_slot_info(gpbs_engine_t* e, int sid, gpbs_slot_info_t* o) {
  LOCK(e);
  Engine& E = *e->e;
  Slot* v = E.slot(sid);
  if (!v) return GPBS_ENOENT;
  std::memset(o, 0, sizeof(*o));
  o->id = v->id;
  o->tenant = v->tenant;
  o->index = v->index;
  o->processor = v->processor;
  o->runstate = v->rs;
  o->is_running = v->is_running;
  for (int i = 0; i < 4; ++i) {
    o->pmc[i] = v->pmc[i];
    o->affinity[i] = v->affinity.w[i];
  }
  o->sched_count = v->sched_count;
  o->class_home = v->class_home;
  o->pause_flags = v->pause_flags;
  const int64_t n = E.now();
  int64_t extra = n - v->rs_entry;
  o->run_ns = v->rs_time[RS_RUNNING] + (v->rs == RS_RUNNING ? extra : 0);
  o->runnable_ns = v->rs_time[RS_RUNNABLE] + (v->rs == RS_RUNNABLE ? extra : 0);
  o->blocked_ns = v->rs_time[RS_BLOCKED] + (v->rs == RS_BLOCKED ? extra : 0);
  if (v->priv)
    if (Scheduler* S = v->is_idle() ? E.sched_of_part(v->processor) : E.sched_of_tenant(v->tenant))
      S->fill_slot_info(*v, *o);
  return GPBS_OK;
}

int gpbs_tenant_adapt_state(gpbs_engine_t* e, int t, gpbs_adapt_state_t* out, int set) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  Scheduler* S = e->e->sched_of_tenant(t);
  AdaptState st;
  if (set) {
    std::memcpy(&st, out, sizeof(st));
    return S->set_tenant_adapt(*d, st) ? GPBS_OK : GPBS_EINVAL;
  }
  if (!S->tenant_adapt(*d, &st)) return GPBS_EINVAL;
  std::memcpy(out, &st, sizeof(st));
  return GPBS_OK;
}

int gpbs_tenant_vpmu(gpbs_engine_t* e, int t, uint64_t* total4) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d || !total4) return GPBS_ENOENT;
  for (int k = 0; k < 4; ++k) total4[k] = d->vpmu_total[k];
  return GPBS_OK;
}

int gpbs_tenant_class(gpbs_engine_t* e, int t) {
  LOCK(e);
  Tenant* d = live(e, t);
  return d ? d->cls : -1;
}

int gpbs_tenant_bound_stats(gpbs_engine_t* e, int t, uint64_t* out3, int reset) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  Scheduler* s = e->e->sched_of_tenant(t);
  return s ? s->bound_stats(*d, out3, reset != 0) : GPBS_EINVAL;
}

int gpbs_tenant_measure(gpbs_engine_t* e, int t, uint32_t us) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  if (us != UINT32_MAX) d->measure_us = us;
  return (int)std::min<uint64_t>(d->measure_granted, INT32_MAX);
}

int gpbs_tenant_switch_cost(gpbs_engine_t* e, int t, uint64_t ns) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  d->sw_cost_us = (uint32_t)std::min<uint64_t>((ns + 500) / 1000, 1000000);
  return GPBS_OK;
}

int gpbs_tenant_slo(gpbs_engine_t* e, int t, uint32_t us) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  if (us > (uint32_t)GPBS_TSLICE_UMAX) return GPBS_ERANGE;
  d->slo_us = us;
  return GPBS_OK;
}

int gpbs_tenant_heartbeat(gpbs_engine_t* e, int t) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  if (e->e->fault(Engine::F_HEARTBEAT_DROP)) return GPBS_OK;  // lost on the way
  d->last_heartbeat = e->e->now();
  return GPBS_OK;
}

int gpbs_sched_credit_get(gpbs_engine_t* e, int t, int* weight, int* cap) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  return e->e->sched_of_tenant(t)->adjust(*d, false, weight, cap);
}

int gpbs_sched_credit_set(gpbs_engine_t* e, int t, int weight, int cap) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  // libxl.c:4026-4045: weight 1..65535, cap 0..100*(max_vcpu_id+1)
  if (weight != -1 && (weight < 1 || weight > GPBS_WEIGHT_MAX)) return GPBS_ERANGE;
  if (cap != -1 && (cap < 0 || cap > 100 * (int)d->slots.size())) return GPBS_ERANGE;
  int r = e->e->sched_of_tenant(t)->adjust(*d, true, &weight, &cap);
  DONE(e);
  return r;
}

// xl sched-credit2 / sched-sedf: scheduler-specific tenant parameters.
int gpbs_sched_ext(gpbs_engine_t* e, int t, int set, gpbs_sched_ext_t* p) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  if (!p) return GPBS_EINVAL;
  int r = e->e->sched_of_tenant(t)->adjust_ext(*d, set != 0, *p);
  if (set) DONE(e);
  return r;
}

int gpbs_arinc653_set(gpbs_engine_t* e, int pool, const gpbs_arinc653_schedule_t* s) {
  LOCK(e);
  Pool* p = e->e->pool(pool);
  if (!p) return GPBS_ENOENT;
  if (!s || s->num_entries < 0 || s->num_entries > GPBS_ARINC653_MAX_ENTRIES) return GPBS_EINVAL;
  std::vector<ArincEntry> es;
  for (int i = 0; i < s->num_entries; ++i) es.push_back({s->entries[i].tenant, s->entries[i].slot, s->entries[i].runtime_ns});
  int r = p->sched->set_schedule(s->major_frame_ns, es);
  DONE(e);
  return r;
}

int gpbs_arinc653_get(gpbs_engine_t* e, int pool, gpbs_arinc653_schedule_t* s) {
  LOCK(e);
  Pool* p = e->e->pool(pool);
  if (!p) return GPBS_ENOENT;
  if (!s) return GPBS_EINVAL;
  int64_t major = 0;
  std::vector<ArincEntry> es;
  int r = p->sched->get_schedule(&major, &es);
  if (r < 0) return r;
  std::memset(s, 0, sizeof(*s));
  s->major_frame_ns = major;
  s->num_entries = (int32_t)std::min<size_t>(es.size(), GPBS_ARINC653_MAX_ENTRIES);
  s->is_explicit = r;
  for (int i = 0; i < s->num_entries; ++i) s->entries[i] = {es[i].tenant, es[i].slot, es[i].runtime};
  return 0;
}

int gpbs_atc_sync(gpbs_engine_t* e, int pool, int global_min_us) {
  LOCK(e);
  Pool* p = e->e->pool(pool);
  if (!p) return GPBS_ENOENT;
  int r = p->sched->atc_sync(global_min_us);
  DONE(e);
  return r;
}

int gpbs_sched_params_get(gpbs_engine_t* e, int pool, int* tslice_us, int* ratelimit_us) {
  LOCK(e);
  Pool* p = e->e->pool(pool);
  if (!p) return GPBS_ENOENT;
  return p->sched->adjust_global(false, tslice_us, ratelimit_us);
}

int gpbs_sched_params_set(gpbs_engine_t* e, int pool, int tslice_us, int ratelimit_us) {
  LOCK(e);
  Pool* p = e->e->pool(pool);
  if (!p) return GPBS_ENOENT;
  int r = p->sched->adjust_global(true, &tslice_us, &ratelimit_us);
  DONE(e);
  return r;
}

int gpbs_sched_name(gpbs_engine_t* e, int pool, char* out, int len) {
  LOCK(e);
  Pool* p = e->e->pool(pool);
  if (!p) return GPBS_ENOENT;
  return copy_str(p->sched->opt_name(), out, len);
}

int gpbs_report_wait(gpbs_engine_t* e, int t, uint64_t wait_ns, int kind) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  e->e->sched_of_tenant(t)->report(*d, wait_ns, kind);
  e->e->perfc.incr(PC_report_rx);
  e->e->emit(TRC_REPORT, 0, t, kind, (uint32_t)wait_ns, (uint32_t)(wait_ns >> 32));
  return GPBS_OK;
}

// Gang window for a tenant (state 0 none, 1 favoured, 2 excluded) until
// `until_ns` on the engine clock; every partition of its pool reschedules now.
int gpbs_gang_set(gpbs_engine_t* e, int t, int state, int64_t until_ns) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d || state < 0 || state > 2) return d ? GPBS_EINVAL : GPBS_ENOENT;
  const int before = d->gang(e->e->now());
  d->gang_state = state;
  d->gang_until = until_ns;
  if (state != before) {
    Pool* pl = e->e->pool(d->pool);
    if (pl)
      for (int p = pl->cpus.first(); p >= 0; p = pl->cpus.next(p + 1)) e->e->raise_softirq(p);
    e->e->perfc.incr(PC_gang_epoch);
    e->e->emit(TRC_GANG_EPOCH, 0, t, (uint32_t)state, (uint32_t)(until_ns / 1000));
  }
  DONE(e);
  return GPBS_OK;
}

int gpbs_report_requests(gpbs_engine_t* e, int t, uint64_t n) {
  LOCK(e);
  Tenant* d = live(e, t);
  if (!d) return GPBS_ENOENT;
  d->pending_requests += n;
  return GPBS_OK;
}

int gpbs_set_counter_ops(gpbs_engine_t* e, const gpbs_counter_ops_t* ops) {
  LOCK(e);
  if (ops)
    e->e->counter_ops = *ops;
  else
    e->e->counter_ops = gpbs_counter_ops_t{};
  return GPBS_OK;
}

int gpbs_set_actuator_ops(gpbs_engine_t* e, const gpbs_actuator_ops_t* ops) {
  LOCK(e);
  if (ops)
    e->e->actuator_ops = *ops;
  else
    e->e->actuator_ops = gpbs_actuator_ops_t{};
  return GPBS_OK;
}

// ---------------------------------------------------- per-GPU backend mux
// The engine lock is held by every caller of these trampolines.
static void mux_on_switch(void* u, int part, int pt, int nt, int ns, int32_t q, int64_t now) {
  Engine* E = (Engine*)u;
  for (auto& m : E->mux)
    if (part >= m.lo && part < m.hi && m.act.on_switch) m.act.on_switch(m.act.user, part, pt, nt, ns, q, now);
}
static void mux_on_flush(void* u, int64_t now) {
  for (auto& m : ((Engine*)u)->mux)
    if (m.act.on_flush) m.act.on_flush(m.act.user, now);
}
static void mux_on_park(void* u, int t, int s, int parked) {
  for (auto& m : ((Engine*)u)->mux)
    if (m.act.on_park) m.act.on_park(m.act.user, t, s, parked);
}
static int mux_slot_refresh(void* u, int sid, int t, int part, uint64_t* pmc) {
  for (auto& m : ((Engine*)u)->mux)
    if (part >= m.lo && part < m.hi && m.ctr.slot_refresh) return m.ctr.slot_refresh(m.ctr.user, sid, t, part, pmc);
  return GPBS_ENOENT;
}
// Node-wide tenant deltas = the sum over the GPUs' backends (the cross-CPU
// pmc gather of X:xen/common/sched_credit.c:416-424).  A backend that fails
// this period contributes nothing; all failing is a stale period.
static int mux_tenant_deltas(void* u, int n, const int* ids, uint64_t* out) {
  Engine* E = (Engine*)u;
  std::vector<uint64_t> part((size_t)4 * n);
  std::fill(out, out + (size_t)4 * n, 0);
  int ok = 0;
  for (auto& m : E->mux) {
    if (!m.ctr.tenant_deltas) continue;
    if (m.ctr.tenant_deltas(m.ctr.user, n, ids, part.data()) != 0) continue;
    ok++;
    for (size_t i = 0; i < part.size(); ++i) out[i] += part[i];
  }
  return ok ? 0 : GPBS_EIO;
}

int gpbs_backend_mux_add(gpbs_engine_t* e, int part_lo, int part_hi, const gpbs_actuator_ops_t* act,
                         const gpbs_counter_ops_t* ctr) {
  LOCK(e);
  if (part_lo < 0 || part_hi <= part_lo) return GPBS_EINVAL;
  Engine* E = e->e;
  for (auto& m : E->mux)
    if (part_lo < m.hi && m.lo < part_hi) return GPBS_EBUSY;  // ranges are disjoint
  Engine::MuxEntry m{part_lo, part_hi, act ? *act : gpbs_actuator_ops_t{}, ctr ? *ctr : gpbs_counter_ops_t{}};
  E->mux.push_back(m);
  gpbs_actuator_ops_t a{};
  a.user = E;
  a.on_switch = mux_on_switch;
  a.on_flush = mux_on_flush;
  a.on_park = mux_on_park;
  E->actuator_ops = a;
  gpbs_counter_ops_t k{};
  k.user = E;
  bool any_refresh = false, any_deltas = false;
  for (auto& x : E->mux) {
    any_refresh |= x.ctr.slot_refresh != nullptr;
    any_deltas |= x.ctr.tenant_deltas != nullptr;
  }
  if (any_refresh) k.slot_refresh = mux_slot_refresh;
  if (any_deltas) k.tenant_deltas = mux_tenant_deltas;
  E->counter_ops = k;
  return (int)E->mux.size() - 1;
}

int gpbs_backend_mux_clear(gpbs_engine_t* e) {
  LOCK(e);
  Engine* E = e->e;
  E->mux.clear();
  E->actuator_ops = gpbs_actuator_ops_t{};
  E->counter_ops = gpbs_counter_ops_t{};
  return GPBS_OK;
}

int gpbs_backend_mux_count(gpbs_engine_t* e) {
  LOCK(e);
  return (int)e->e->mux.size();
}

int gpbs_get_actuator_ops(gpbs_engine_t* e, gpbs_actuator_ops_t* out) {
  LOCK(e);
  *out = e->e->actuator_ops;
  return GPBS_OK;
}

int gpbs_get_counter_ops(gpbs_engine_t* e, gpbs_counter_ops_t* out) {
  LOCK(e);
  *out = e->e->counter_ops;
  return GPBS_OK;
}

int gpbs_slot_set_pmc(gpbs_engine_t* e, int sid, const uint64_t* pmc4) {
  LOCK(e);
  Slot* v = e->e->slot(sid);
  if (!v) return GPBS_ENOENT;
  for (int i = 0; i < 4; ++i) v->pmc[i] = pmc4[i];
  return GPBS_OK;
}

int64_t gpbs_now(gpbs_engine_t* e) { return e->e->now(); }

int gpbs_advance(gpbs_engine_t* e, int64_t now_ns) {
  LOCK(e);
  if (!e->e->boot.sim_clock) return GPBS_EINVAL;
  e->e->run_due(now_ns);
  return GPBS_OK;
}

int gpbs_start(gpbs_engine_t* e) { return e->e->start(); }
int gpbs_stop(gpbs_engine_t* e) { return e->e->stop(); }

int gpbs_poll(gpbs_engine_t* e) {
  LOCK(e);
  e->e->run_due(e->e->now());
  return GPBS_OK;
}

int64_t gpbs_next_event(gpbs_engine_t* e) {
  LOCK(e);
  return e->e->next_deadline();
}

int gpbs_debug_keys(gpbs_engine_t* e, const char* keys, char* out, int len) {
  LOCK(e);
  return copy_str(e->e->debug_keys(keys ? keys : ""), out, len);
}

int gpbs_dmesg(gpbs_engine_t* e, char* out, int len, int clear) {
  LOCK(e);
  return copy_str(e->e->dmesg(clear != 0), out, len);
}

int gpbs_trace_read(gpbs_engine_t* e, uint64_t* cursor, gpbs_trace_record_t* out, int max, uint64_t* lost) {
  return (int)e->e->trace->read(cursor, reinterpret_cast<TraceRecord*>(out), (size_t)max, lost);
}

int gpbs_trace_set_mask(gpbs_engine_t* e, uint64_t mask) {
  e->e->trace->set_mask(mask);
  return GPBS_OK;
}

int gpbs_trace_emit(gpbs_engine_t* e, uint32_t ev, uint32_t cpu, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
  LOCK(e);
  e->e->emit(ev, cpu, a0, a1, a2, a3);
  if (ev == TRC_GANG_EPOCH) e->e->perfc.incr(PC_gang_epoch);
  return GPBS_OK;
}

int gpbs_perfc_count(void) { return PC_COUNT; }
const char* gpbs_perfc_name(int i) { return i >= 0 && i < PC_COUNT ? kPerfcNames[i] : nullptr; }

int gpbs_perfc_read(gpbs_engine_t* e, uint64_t* out, int max) {
  int n = std::min(max, (int)PC_COUNT);
  for (int i = 0; i < n; ++i) out[i] = e->e->perfc.get((PerfcId)i);
  return n;
}

int gpbs_perfc_reset(gpbs_engine_t* e) {
  e->e->perfc.reset();
  return GPBS_OK;
}

int gpbs_check_invariants(gpbs_engine_t* e, char* out, int len) {
  LOCK(e);
  std::string s = e->e->check_invariants();
  copy_str(s, out, len);
  return s.empty() ? 0 : 1;
}

int gpbs_lockprof(gpbs_engine_t* e, gpbs_lockprof_t* out, int reset) {
  LockProfile& p = e->e->lockprof;
  if (out) {
    out->lock_cnt = p.lock_cnt.load();
    out->block_cnt = p.block_cnt.load();
    out->time_block_ns = p.time_block_ns.load();
    out->time_hold_ns = p.time_hold_ns.load();
    out->max_block_ns = p.max_block_ns.load();
    out->max_hold_ns = p.max_hold_ns.load();
    out->handoffs = p.handoffs.load();
  }
  if (reset) p.reset();
  return GPBS_OK;
}

int gpbs_watchdog(gpbs_engine_t* e, int tenant, uint32_t id, uint32_t timeout_ms) {
  LOCK(e);
  int rc = e->e->watchdog(tenant, id, timeout_ms);
  DONE(e);
  return rc;
}

}  // extern "C"

// Host reference adaptation exposed for oracle/device parity tests.
extern "C" void gpbs_adapt_init(gpbs_adapt_state_t* s, const gpbs_adapt_params_t* p, uint32_t default_tslice_us) {
  adapt_init(*reinterpret_cast<AdaptState*>(s), *reinterpret_cast<const AdaptParams*>(p), default_tslice_us);
}

extern "C" int gpbs_adapt_update(gpbs_adapt_state_t* s, const gpbs_adapt_params_t* p, uint64_t inst, uint64_t miss,
                                 uint64_t spin_sum, uint64_t spin_cnt) {
  bool rearm = false;
  int d = adapt_update(*reinterpret_cast<AdaptState*>(s), *reinterpret_cast<const AdaptParams*>(p), inst, miss,
                       spin_sum, spin_cnt, &rearm);
  return (d + 1) | (rearm ? 4 : 0);
}
