// Host-CPU counter backend: perf_event_open with the
// same four events PBS reads through Perfctr-xen -- instructions retired,
// unhalted cycles, LLC references, LLC misses (X:xen/common/sched_credit.c:1966
// labels; X:xen/arch/x86/perfctr.c:1547-1572 is the per-vCPU save it replaces).
// One counter set per tenant process (inherit=1: its threads and children).
//
// Containers and VMs often expose no hardware PMU.  Then the set degrades to
// software events, reported by gpbs_perf_mode(): task-clock stands in for both
// instructions and cycles (IPC 1), minor/major page faults for LLC
// references/misses -- enough to drive the plumbing, not a miss-rate signal.
#include <linux/perf_event.h>
#include <sys/ioctl.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstring>

#include "../include/gpbs/gpbs.h"

namespace {

struct PerfSet {
  int fd[4] = {-1, -1, -1, -1};
  int mode = 0;  // GPBS_PERF_HW / GPBS_PERF_SW
};

long perf_open(perf_event_attr* a, int pid, int cpu) {
  return syscall(SYS_perf_event_open, a, pid, cpu, -1, 0);
}

int open_one(uint32_t type, uint64_t config, int pid, int cpu) {
  perf_event_attr a;
  std::memset(&a, 0, sizeof(a));
  a.size = sizeof(a);
  a.type = type;
  a.config = config;
  a.inherit = 1;
  a.exclude_kernel = 1;  // perf_event_paranoid <= 2 allows user-only counting
  a.exclude_hv = 1;
  a.read_format = PERF_FORMAT_TOTAL_TIME_ENABLED | PERF_FORMAT_TOTAL_TIME_RUNNING;
  return (int)perf_open(&a, pid, cpu);
}

void close_all(PerfSet* s) {
  for (int& f : s->fd)
    if (f >= 0) {
      close(f);
      f = -1;
    }
}

}  // namespace

extern "C" {

void* gpbs_perf_open(int pid, int cpu) {
  auto* s = new PerfSet;
  const uint64_t hw[4] = {PERF_COUNT_HW_INSTRUCTIONS, PERF_COUNT_HW_CPU_CYCLES, PERF_COUNT_HW_CACHE_REFERENCES,
                          PERF_COUNT_HW_CACHE_MISSES};
  bool ok = true;
  for (int i = 0; i < 4 && ok; ++i) ok = (s->fd[i] = open_one(PERF_TYPE_HARDWARE, hw[i], pid, cpu)) >= 0;
  if (ok) {
    s->mode = GPBS_PERF_HW;
    return s;
  }
  close_all(s);
  const uint64_t sw[4] = {PERF_COUNT_SW_TASK_CLOCK, PERF_COUNT_SW_TASK_CLOCK, PERF_COUNT_SW_PAGE_FAULTS_MIN,
                          PERF_COUNT_SW_PAGE_FAULTS_MAJ};
  ok = true;
  for (int i = 0; i < 4 && ok; ++i) ok = (s->fd[i] = open_one(PERF_TYPE_SOFTWARE, sw[i], pid, cpu)) >= 0;
  if (ok) {
    s->mode = GPBS_PERF_SW;
    return s;
  }
  close_all(s);
  delete s;
  return nullptr;
}

// Cumulative values, scaled for multiplexing (time_enabled / time_running).
int gpbs_perf_read(void* h, uint64_t* out4) {
  auto* s = (PerfSet*)h;
  if (!s || !out4) return GPBS_EINVAL;
  for (int i = 0; i < 4; ++i) {
    uint64_t v[3] = {0, 0, 0};
    if (read(s->fd[i], v, sizeof(v)) != (ssize_t)sizeof(v)) return GPBS_EIO;
    out4[i] = (v[2] && v[2] < v[1]) ? (uint64_t)((double)v[0] * ((double)v[1] / (double)v[2])) : v[0];
  }
  return GPBS_OK;
}

int gpbs_perf_mode(void* h) { return h ? ((PerfSet*)h)->mode : 0; }

void gpbs_perf_close(void* h) {
  auto* s = (PerfSet*)h;
  if (!s) return;
  close_all(s);
  delete s;
}

// What this host supports for the calling process: GPBS_PERF_HW, GPBS_PERF_SW or 0.
int gpbs_perf_available(void) {
  void* h = gpbs_perf_open(0, -1);
  const int m = gpbs_perf_mode(h);
  gpbs_perf_close(h);
  return m;
}

}  // extern "C"
