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
// Layout: header, then per rank {seq, want, vals[2][kMaxVals]}.  A rank writes
// its values for epoch e into vals[e & 1], then publishes seq = e (release).
// It cannot reach epoch e + 2 before every member has published e + 1, so a
// slow reader of vals[e & 1] is never overwritten.
//
// Views (elastic re-formation, the analog of the reference moving the pool
// master's timers to a surviving CPU, X:xen/common/sched_credit.c:628-633):
// the gang starts as view 0 = every rank.  After a missed deadline the
// survivors call gpbs_gang_shm_reform: the first one to claim generation g
// becomes the master of the re-formation, waits a join window, and publishes
// view g = the ranks that asked to join g (members mask) with a common first
// epoch.  Exchanges then wait only for members.  A rank that was left out --
// the hung one when it comes back -- finds the view changed under it and
// gets -116 (ESTALE) from its next exchange instead of reading epochs that
// are not its own.  It may ask to rejoin (a re-formation it claims); the
// members see the newer claim at their next exchange (-117) and join it.  A
// rank dropped kMaxStrikes times stays out: a rank that keeps hanging would
// otherwise cost the gang a deadline per cycle.
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
#include <algorithm>

namespace {

constexpr int kMaxRanks = 64;
constexpr int kMaxVals = 128;

constexpr uint32_t kMaxStrikes = 2;  // exclusions after which a rank may not rejoin

struct alignas(64) RankSlot {
  std::atomic<uint64_t> seq;
  std::atomic<uint64_t> want;     // view generation this rank asked to join
  std::atomic<uint32_t> strikes;  // times a published view dropped this rank
  int64_t vals[2][kMaxVals];
};

struct Region {
  std::atomic<uint32_t> magic;
  uint32_t world, nvals, pad;
  std::atomic<uint64_t> claim;         // highest generation a master claimed
  std::atomic<uint64_t> view_gen;      // published view (0 = every rank)
  std::atomic<uint64_t> view_members;  // member mask of view_gen (0 in view 0 = all)
  std::atomic<uint64_t> view_base;     // first epoch of view_gen
  RankSlot ranks[kMaxRanks];
};

struct Gang {
  Region* r = nullptr;
  size_t size = 0;
  int fd = -1;
  int rank = 0, world = 1, nvals = 0;
  uint64_t gen = 0, members = 0;  // this rank's view
  std::string name;
};

uint64_t all_mask(int world) { return world >= 64 ? ~0ull : ((1ull << world) - 1); }

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
  g->members = all_mask(world);
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
  if (g->r->view_gen.load(std::memory_order_acquire) != g->gen) return -116;  // re-formed without us
  if (g->r->claim.load(std::memory_order_acquire) > g->gen) return -117;     // a newer view is forming: join it
  RankSlot& me = g->r->ranks[g->rank];
  const int buf = (int)(epoch & 1);
  std::memcpy(me.vals[buf], in, sizeof(int64_t) * g->nvals);
  me.seq.store(epoch, std::memory_order_release);
  for (int k = 0; k < g->world; ++k) {
    if (!((g->members >> k) & 1)) continue;
    RankSlot& o = g->r->ranks[k];
    int spins = 0;
    while (o.seq.load(std::memory_order_acquire) < epoch) {
      // the peers normally arrive within microseconds: busy-poll first
      // (PAUSE), then yield, then sleep until the deadline.  The deadline is
      // checked in every phase: on a loaded host one sched_yield can give
      // the CPU away for a whole time slice, and 256 of them overran a
      // 200 ms deadline by up to 0.5 s (tests/test_gang_deadline.py under
      // pytest -n 4)
      ++spins;
      if (spins < 4096) {
        __builtin_ia32_pause();
        if ((spins & 255) == 0 && now_ns() > deadline_ns) return -110;
        continue;
      }
      if (now_ns() > deadline_ns) return -110;
      if (spins < 4096 + 256) {
        std::this_thread::yield();
        continue;
      }
      if (g->r->view_gen.load(std::memory_order_acquire) != g->gen) return -116;
      if (g->r->claim.load(std::memory_order_acquire) > g->gen) return -117;
      timespec ts{0, 2000};  // 2 us
      nanosleep(&ts, nullptr);
    }
    std::memcpy(out + (size_t)k * g->nvals, o.vals[buf], sizeof(int64_t) * g->nvals);
  }
  // a view published while we gathered may have started from other epochs
  if (g->r->view_gen.load(std::memory_order_acquire) != g->gen) return -116;
  return 0;
}

// Elastic re-formation after a missed deadline (see the header comment).
// Every survivor calls this; the first to claim the next generation waits
// `join_ns` for the others to ask, then publishes the view.  Returns 0 with
// *members (mask over the original ranks) and *base_epoch (the first epoch
// every member uses next) when this rank is a member, -1 when the view was
// published without it, -110 when no view appeared by `deadline_ns`.
int gpbs_gang_shm_reform(void* h, int64_t join_ns, int64_t deadline_ns, uint64_t* members, uint64_t* base_epoch) {
  Gang* g = (Gang*)h;
  if (!g) return -22;
  Region* R = g->r;
  if (R->ranks[g->rank].strikes.load(std::memory_order_acquire) >= kMaxStrikes) return -1;
  // join the generation being formed, or claim the next one
  const uint64_t vg0 = R->view_gen.load(std::memory_order_acquire);
  const uint64_t cl0 = R->claim.load(std::memory_order_acquire);
  const uint64_t want = cl0 > vg0 ? cl0 : vg0 + 1;
  R->ranks[g->rank].want.store(want, std::memory_order_release);
  uint64_t expect = want - 1;
  if (R->claim.compare_exchange_strong(expect, want, std::memory_order_acq_rel)) {
    // master of this re-formation: wait until every rank that published the
    // epoch we timed out on (it is alive, and will time out too) has asked
    // to join, or the join window closes; the laggard that never published
    // that epoch is not waited for
    const uint64_t mine = R->ranks[g->rank].seq.load(std::memory_order_acquire);
    const int64_t close_at = now_ns() + join_ns;
    while (now_ns() < close_at) {
      bool all = true;
      for (int k = 0; k < g->world && all; ++k)
        if (R->ranks[k].seq.load(std::memory_order_acquire) >= mine)
          all = R->ranks[k].want.load(std::memory_order_acquire) >= want;
      if (all) break;
      timespec ts{0, 200000};  // 200 us
      nanosleep(&ts, nullptr);
    }
    uint64_t m = 0, base = 0;
    for (int k = 0; k < g->world; ++k)
      if (R->ranks[k].want.load(std::memory_order_acquire) >= want) {
        m |= 1ull << k;
        base = std::max<uint64_t>(base, R->ranks[k].seq.load(std::memory_order_acquire));
      }
    const uint64_t prev_gen = R->view_gen.load(std::memory_order_acquire);
    const uint64_t prev = prev_gen ? R->view_members.load(std::memory_order_relaxed) : all_mask(g->world);
    for (int k = 0; k < g->world; ++k)
      if (((prev >> k) & 1) && !((m >> k) & 1)) R->ranks[k].strikes.fetch_add(1, std::memory_order_acq_rel);
    R->view_members.store(m, std::memory_order_relaxed);
    R->view_base.store(base + 2, std::memory_order_relaxed);
    R->view_gen.store(want, std::memory_order_release);
  } else {
    while (R->view_gen.load(std::memory_order_acquire) < want) {
      if (now_ns() > deadline_ns) return -110;
      timespec ts{0, 200000};
      nanosleep(&ts, nullptr);
    }
  }
  const uint64_t vg = R->view_gen.load(std::memory_order_acquire);
  const uint64_t m = R->view_members.load(std::memory_order_relaxed);
  if (vg != want || !((m >> g->rank) & 1)) return -1;
  g->gen = vg;
  g->members = m;
  if (members) *members = m;
  if (base_epoch) *base_epoch = R->view_base.load(std::memory_order_relaxed);
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
