// Host-CPU actuation backend: the engine's
// partitions are host CPUs and its tenants are Linux processes.  A partition
// switch (X:xen/common/schedule.c:1082-1185 context_switch analog) updates the
// set of CPUs each tenant holds; a tenant holding none is stopped (SIGSTOP),
// otherwise it is continued (SIGCONT) and every thread is pinned to exactly
// its CPUs (sched_setaffinity) -- the vCPU -> pCPU mapping made literal.
//
// gpbs_cpu_backend_* binds a gate and per-tenant perf_event counter sets to an
// engine: actuator on_switch/on_flush drive the gate, counter slot_refresh
// publishes the tenant's cumulative counters on its slot 0 (the per-domain
// reduction of X:xen/common/sched_credit.c:416-424 sums over slots).
#include <dirent.h>
#include <sched.h>
#include <signal.h>
#include <sys/types.h>

#include <cstdint>
#include <cstdlib>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../include/gpbs/gpbs.h"

extern "C" {
void* gpbs_perf_open(int pid, int cpu);
int gpbs_perf_read(void* h, uint64_t* out4);
void gpbs_perf_close(void* h);
}

namespace {

struct Gate {
  std::mutex mu;
  std::map<int, std::vector<int>> pids;      // tenant -> processes
  std::map<int, std::set<int>> cpus;         // tenant -> host CPUs held now
  std::map<int, bool> stopped;               // tenant -> SIGSTOPped
  std::set<int> dirty;
  uint64_t signals = 0, pins = 0;
};

void pin_all_threads(int pid, const std::set<int>& cpus) {
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus) CPU_SET(c, &set);
  const std::string dir = "/proc/" + std::to_string(pid) + "/task";
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* e = readdir(d)) {
      const int tid = atoi(e->d_name);
      if (tid > 0) sched_setaffinity(tid, sizeof(set), &set);
    }
    closedir(d);
  } else {
    sched_setaffinity(pid, sizeof(set), &set);
  }
}

void apply(Gate* g, int t) {
  const auto& cs = g->cpus[t];
  const bool stop = cs.empty();
  for (int pid : g->pids[t]) {
    if (!stop) {
      pin_all_threads(pid, cs);
      g->pins++;
    }
    if (stop != g->stopped[t]) {
      kill(pid, stop ? SIGSTOP : SIGCONT);
      g->signals++;
    }
  }
  g->stopped[t] = stop;
}

struct Backend {
  gpbs_engine_t* engine = nullptr;
  Gate* gate = nullptr;
  std::map<int, int> host_cpu;               // partition -> host CPU
  std::map<int, void*> perf;                 // tenant -> counter set
  std::map<int, int> part_tenant;            // partition -> tenant running now
  gpbs_actuator_ops_t chained{};
};

void be_on_switch(void* user, int part, int prev, int next, int slot, int32_t q, int64_t now) {
  auto* b = (Backend*)user;
  if (b->chained.on_switch) b->chained.on_switch(b->chained.user, part, prev, next, slot, q, now);
  auto it = b->host_cpu.find(part);
  if (it == b->host_cpu.end()) return;
  std::lock_guard<std::mutex> g(b->gate->mu);
  if (prev >= 0) {
    b->gate->cpus[prev].erase(it->second);
    b->gate->dirty.insert(prev);
  }
  if (next >= 0) {
    b->gate->cpus[next].insert(it->second);
    b->gate->dirty.insert(next);
  }
  b->part_tenant[part] = next;
}

// One batch of engine work -> one signal/pin pass per touched tenant (a
// tenant moving between CPUs is never stopped in between).
void be_on_flush(void* user, int64_t now) {
  auto* b = (Backend*)user;
  if (b->chained.on_flush) b->chained.on_flush(b->chained.user, now);
  std::lock_guard<std::mutex> g(b->gate->mu);
  for (int t : b->gate->dirty)
    if (b->gate->pids.count(t)) apply(b->gate, t);
  b->gate->dirty.clear();
}

int be_slot_refresh(void* user, int slot_id, int tenant, int part, uint64_t* pmc) {
  (void)slot_id;
  (void)part;
  auto* b = (Backend*)user;
  auto it = b->perf.find(tenant);
  if (it == b->perf.end() || !it->second) return 0;
  // Only slot 0 carries the process-wide counters: the per-domain delta sums
  // slots, so publishing on every slot would count the process n times.
  int idx = -1;
  gpbs_slot_info_t si;
  if (gpbs_slot_info(b->engine, slot_id, &si) == GPBS_OK) idx = si.index;
  if (idx != 0) return 0;
  uint64_t v[4];
  if (gpbs_perf_read(it->second, v) != GPBS_OK) return 0;
  for (int i = 0; i < 4; ++i) pmc[i] = v[i];
  return 0;
}

}  // namespace

extern "C" {

void* gpbs_gate_create(const char* mode) {
  if (mode && *mode && std::string(mode) != "signal") return nullptr;  // cgroup mode: not built
  return new Gate;
}

int gpbs_gate_mode(void* g) { return g ? 1 : 0; }  // 1 = signal + affinity

int gpbs_gate_add_pid(void* gp, int tenant, int pid) {
  auto* g = (Gate*)gp;
  if (!g || pid <= 0) return GPBS_EINVAL;
  std::lock_guard<std::mutex> l(g->mu);
  g->pids[tenant].push_back(pid);
  g->dirty.insert(tenant);
  return GPBS_OK;
}

// Direct control (tests / manual mode): give or take one host CPU.
int gpbs_gate_set(void* gp, int tenant, int cpu, int on) {
  auto* g = (Gate*)gp;
  if (!g) return GPBS_EINVAL;
  std::lock_guard<std::mutex> l(g->mu);
  if (on)
    g->cpus[tenant].insert(cpu);
  else
    g->cpus[tenant].erase(cpu);
  apply(g, tenant);
  return GPBS_OK;
}

int gpbs_gate_stats(void* gp, uint64_t* signals, uint64_t* pins) {
  auto* g = (Gate*)gp;
  if (!g) return GPBS_EINVAL;
  std::lock_guard<std::mutex> l(g->mu);
  if (signals) *signals = g->signals;
  if (pins) *pins = g->pins;
  return GPBS_OK;
}

// Release every tenant (SIGCONT, all CPUs) and free the gate.
void gpbs_gate_destroy(void* gp) {
  auto* g = (Gate*)gp;
  if (!g) return;
  {
    std::lock_guard<std::mutex> l(g->mu);
    for (auto& kv : g->pids)
      for (int pid : kv.second) kill(pid, SIGCONT);
  }
  delete g;
}

void* gpbs_cpu_backend_create(gpbs_engine_t* e, void* gate) {
  if (!e || !gate) return nullptr;
  auto* b = new Backend;
  b->engine = e;
  b->gate = (Gate*)gate;
  gpbs_get_actuator_ops(e, &b->chained);
  gpbs_actuator_ops_t a{};
  a.user = b;
  a.on_switch = be_on_switch;
  a.on_flush = be_on_flush;
  a.on_park = b->chained.on_park;
  gpbs_set_actuator_ops(e, &a);
  gpbs_counter_ops_t c{};
  c.user = b;
  c.slot_refresh = be_slot_refresh;
  gpbs_set_counter_ops(e, &c);
  return b;
}

int gpbs_cpu_backend_map(void* bp, int partition, int host_cpu) {
  auto* b = (Backend*)bp;
  if (!b || partition < 0 || host_cpu < 0) return GPBS_EINVAL;
  b->host_cpu[partition] = host_cpu;
  return GPBS_OK;
}

// Register a tenant process: counters (perf_event, inherit) + gate.  The
// process starts stopped until the engine gives the tenant a CPU.
int gpbs_cpu_backend_add(void* bp, int tenant, int pid) {
  auto* b = (Backend*)bp;
  if (!b || pid <= 0) return GPBS_EINVAL;
  if (!b->perf.count(tenant)) b->perf[tenant] = gpbs_perf_open(pid, -1);
  int rc = gpbs_gate_add_pid(b->gate, tenant, pid);
  if (rc) return rc;
  std::lock_guard<std::mutex> l(b->gate->mu);
  apply(b->gate, tenant);
  return b->perf[tenant] ? GPBS_OK : GPBS_ENOENT;  // ENOENT: gated, but no counters
}

void gpbs_cpu_backend_destroy(void* bp) {
  auto* b = (Backend*)bp;
  if (!b) return;
  gpbs_set_actuator_ops(b->engine, b->chained.on_switch || b->chained.on_flush ? &b->chained : nullptr);
  gpbs_set_counter_ops(b->engine, nullptr);
  for (auto& kv : b->perf) gpbs_perf_close(kv.second);
  delete b;
}

}  // extern "C"
