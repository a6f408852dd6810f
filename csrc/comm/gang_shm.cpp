// Node-local gang epoch transport over POSIX shared memory (SURVEY §2.6 C16,
// §2.8 (b)): the per-GPU scheduler ranks of one node (one process per GPU)
// meet at every gang epoch and all-gather a few int64 values -- per gang
// tenant "has demand here", the ATC slice, the keep-going flag, the previous
// epoch's return time -- with a deadline.
//
// The message is tens of bytes and latency-bound; all eight ranks of an
// MI355X node share one host, so the barrier is a seqlock-style slot per rank
// in one shm region (no kernel launch, no CU time, no xGMI traffic next to
// the tenants' own RCCL all-reduce), ~microseconds instead of the tens of
// microseconds of an RCCL or gloo collective (scripts/gang_bench.py).  A rank
// that misses the deadline makes the call return -110 (ETIMEDOUT) on every
// other rank: they degrade to local scheduling instead of stalling (§5.3).
//
// Layout: header, then per rank {seq, vals[2][kMaxVals]}.  A rank writes its
// values for epoch e into vals[e & 1], then publishes seq = e (release).  It
// cannot reach epoch e + 2 before every rank has published e + 1, so a slow
// reader of vals[e & 1] is never overwritten.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>

namespace {

constexpr int kMaxRanks = 64;
constexpr int kMaxVals = 128;

struct alignas(64) RankSlot {
  std::atomic<uint64_t> seq;
  int64_t vals[2][kMaxVals];
};

struct Region {
  std::atomic<uint32_t> magic;
  uint32_t world, nvals, pad;
  RankSlot ranks[kMaxRanks];
};

struct Gang {
  Region* r = nullptr;
  size_t size = 0;
  int fd = -1;
  int rank = 0, world = 1, nvals = 0;
  std::string name;
};

int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000ll + ts.tv_nsec;
}

}  // namespace

extern "C" {

// Open (creating if needed) the region `name` for `world` ranks exchanging
// `nvals` int64 per epoch.  Every rank must use the same fresh name (the
// caller agrees on a nonce); rank 0 unlinks it at close.
void* gpbs_gang_shm_open(const char* name, int rank, int world, int nvals) {
  if (!name || world < 1 || world > kMaxRanks || rank < 0 || rank >= world || nvals < 0 || nvals > kMaxVals)
    return nullptr;
  auto* g = new Gang;
  g->name = name[0] == '/' ? name : std::string("/") + name;
  g->rank = rank;
  g->world = world;
  g->nvals = nvals;
  g->size = sizeof(Region);
  g->fd = shm_open(g->name.c_str(), O_CREAT | O_RDWR, 0600);
  if (g->fd < 0 || ftruncate(g->fd, (off_t)g->size) != 0) {
    if (g->fd >= 0) close(g->fd);
    delete g;
    return nullptr;
  }
  void* p = mmap(nullptr, g->size, PROT_READ | PROT_WRITE, MAP_SHARED, g->fd, 0);
  if (p == MAP_FAILED) {
    close(g->fd);
    delete g;
    return nullptr;
  }
  g->r = (Region*)p;  // zero-filled on creation: every seq starts at 0, epochs at 1
  return g;
}

// All-gather `in[nvals]` of every rank for `epoch` (1, 2, ...; strictly
// increasing per rank, one per call) into out[world * nvals] (rank-major);
// the caller reduces (MIN for the window vector, SUM for node metrics).
// Returns 0, -110 when some rank had not arrived by `deadline_ns`
// (CLOCK_MONOTONIC), or -22.
int gpbs_gang_shm_allgather(void* h, uint64_t epoch, const int64_t* in, int64_t* out, int64_t deadline_ns) {
  Gang* g = (Gang*)h;
  if (!g || !epoch || (g->nvals && (!in || !out))) return -22;
  RankSlot& me = g->r->ranks[g->rank];
  const int buf = (int)(epoch & 1);
  std::memcpy(me.vals[buf], in, sizeof(int64_t) * g->nvals);
  me.seq.store(epoch, std::memory_order_release);
  for (int k = 0; k < g->world; ++k) {
    RankSlot& o = g->r->ranks[k];
    int spins = 0;
    while (o.seq.load(std::memory_order_acquire) < epoch) {
      // the peers normally arrive within microseconds: busy-poll first
      // (PAUSE), then yield, then sleep until the deadline
      if (++spins < 4096) {
        __builtin_ia32_pause();
        continue;
      }
      if (spins < 4096 + 256) {
        std::this_thread::yield();
        continue;
      }
      if (now_ns() > deadline_ns) return -110;
      timespec ts{0, 2000};  // 2 us
      nanosleep(&ts, nullptr);
    }
    std::memcpy(out + (size_t)k * g->nvals, o.vals[buf], sizeof(int64_t) * g->nvals);
  }
  return 0;
}

void gpbs_gang_shm_close(void* h) {
  Gang* g = (Gang*)h;
  if (!g) return;
  munmap(g->r, g->size);
  close(g->fd);
  if (g->rank == 0) shm_unlink(g->name.c_str());
  delete g;
}

}  // extern "C"
