// Tenant <-> scheduler shared-memory control plane (replaces the reference's
// hypercall page, shared_info pages and VIRQ upcalls):
//
//  * one 4 KiB page per tenant in a POSIX shm region "/gpbs-<name>";
//  * scheduler -> tenant assignment words under a seqlock (the reader retries
//    like the Perfctr-xen paravirtual counter read, L:drivers/perfctr/x86.c:252-277);
//  * tenant -> scheduler: heartbeat, has-work flag, cumulative software
//    counters (vPMU mirror, C10) and an SPSC ring of wait reports
//    {u64 wait_ns, u32 kind, u32 gpu} (the vcrd_op hypercall, C7);
//  * a futex doorbell per page (VIRQ analog, C9/C1) so gated tenants sleep;
//  * scheduler -> tenant vPMU mirror under its own seqlock: the cumulative
//    counters the scheduler measured (live CDNA4 counters attributed by
//    ownership, or the tenant's own declared ones) plus the PBS view of the
//    tenant (miss rate, quantum, class, phase) -- the Perfctr-xen per-vCPU
//    state page the guest reads with a version check (S1/S2, C10, K13).
//
// The bridge thread binds a region to an engine: it turns page traffic into
// engine calls (wake/block, report_wait, heartbeat, slot pmc) and publishes
// engine switches back into the pages (chaining any actuator already set,
// e.g. the GPU partition-table actuator).
#include <fcntl.h>
#include <linux/futex.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../include/gpbs/gpbs.h"

namespace {

constexpr uint32_t kMagic = 0x53425047;  // "GPBS"
constexpr uint32_t kVersion = 2;  // 2: vPMU mirror block
constexpr int kRing = 192;

struct Report {
  uint64_t wait_ns;
  uint32_t kind;
  uint32_t gpu;
};

struct alignas(64) Page {
  // ---- scheduler -> tenant (seqlock: seq odd while writing)
  // Payload words are relaxed atomics: the seqlock orders them, the atomics
  // make the concurrent (retried) reads well-defined.
  std::atomic<uint32_t> seq;
  std::atomic<uint32_t> gate;        // 1: may launch, 0: gated (no partition / parked / paused)
  std::atomic<uint64_t> mask[2];     // partitions currently running the tenant (bit = partition id, < 128)
  std::atomic<uint32_t> quantum_us;
  std::atomic<int32_t> priority;     // stream priority hint: 1 high (BOOST), 0 normal
  std::atomic<int32_t> tenant_id;    // engine tenant id (-1: unused page)
  std::atomic<uint32_t> epoch;
  uint8_t pad0[64 - 40];
  // ---- tenant -> scheduler
  std::atomic<uint64_t> heartbeat_ns;
  std::atomic<uint32_t> has_work;
  std::atomic<uint32_t> progress;
  std::atomic<uint64_t> counters[4];
  std::atomic<int32_t> pid;
  uint8_t pad1[64 - 52];
  // ---- SPSC report ring (tenant produces, bridge consumes)
  std::atomic<uint32_t> rhead;
  std::atomic<uint32_t> rtail;
  std::atomic<uint32_t> dropped;
  std::atomic<uint32_t> doorbell;  // futex word, bumped on every publish that opens the gate
  uint8_t pad2[64 - 16];
  // ---- scheduler -> tenant vPMU mirror (seqlock vseq, odd while writing)
  std::atomic<uint32_t> vseq;
  std::atomic<uint32_t> vphase;
  std::atomic<uint64_t> vpmu[4];     // cumulative INST, CYCLES, LLC refs, LLC misses
  std::atomic<uint64_t> vmiss_rate;  // last period, per 100k instructions
  std::atomic<uint32_t> vtslice_us;
  std::atomic<int32_t> vclass;
  uint8_t pad3[64 - 56];
  Report ring[kRing];
};
static_assert(sizeof(Page) <= 4096, "ctl page exceeds 4 KiB");

struct Header {
  uint32_t magic, version, ntenants, page_size;
  std::atomic<uint64_t> epoch;
  uint8_t pad[4096 - 24];
};

struct Ctl {
  std::string name;
  int fd = -1;
  size_t size = 0;
  Header* hdr = nullptr;
  Page* pages = nullptr;
  bool owner = false;
  // bridge
  gpbs_engine_t* engine = nullptr;
  gpbs_actuator_ops_t chained{};
  std::vector<uint64_t> pend_mask;  // per tenant id x 2 words
  std::vector<uint32_t> last_work;
  std::vector<uint32_t> last_hb_sent;
  std::thread th;
  std::atomic<bool> stop{false};
  std::mutex mu;
  std::mutex pub_mu;  // one seqlock writer at a time (flush vs. assign/publish)
  uint32_t epoch = 0;
  // torn_page fault: a publish left half-written (seq odd) that the bridge
  // thread completes at `due` -- never a sleep under the engine lock
  struct Torn {
    bool active = false;
    int64_t due = 0;
    uint64_t mask1 = 0;
    uint32_t quantum = 0, epoch = 0, seq = 0, gate = 0, old_gate = 0;
    int32_t prio = 0, tid = -1;
  };
  std::vector<Torn> torn;  // per page (pub_mu)
};

int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000ll + ts.tv_nsec;
}

long futex(std::atomic<uint32_t>* a, int op, uint32_t val, const timespec* to) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(a), op, val, to, nullptr, 0);
}

Page* page(void* h, int t) {
  Ctl* c = (Ctl*)h;
  if (!c || t < 0 || t >= (int)c->hdr->ntenants) return nullptr;
  return &c->pages[t];
}

Ctl* map_region(const char* name, int ntenants, bool create) {
  std::string n = std::string("/gpbs-") + name;
  // O_EXCL: never truncate a region another live daemon (or this process) maps
  // -- that would SIGBUS every tenant holding the old mapping.
  int fd = create ? shm_open(n.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600) : shm_open(n.c_str(), O_RDWR, 0);
  if (fd < 0) return nullptr;
  size_t size;
  if (create) {
    size = sizeof(Header) + (size_t)ntenants * 4096;
    if (ftruncate(fd, (off_t)size) != 0) {
      close(fd);
      return nullptr;
    }
  } else {
    struct stat st;
    if (fstat(fd, &st) != 0) {
      close(fd);
      return nullptr;
    }
    size = (size_t)st.st_size;
  }
  void* p = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    close(fd);
    return nullptr;
  }
  auto* c = new Ctl;
  c->name = n;
  c->fd = fd;
  c->size = size;
  c->hdr = (Header*)p;
  c->pages = (Page*)((char*)p + sizeof(Header));
  c->owner = create;
  if (create) {
    std::memset(p, 0, size);
    c->hdr->magic = kMagic;
    c->hdr->version = kVersion;
    c->hdr->ntenants = (uint32_t)ntenants;
    c->hdr->page_size = 4096;
    for (int t = 0; t < ntenants; ++t) c->pages[t].tenant_id.store(-1, std::memory_order_relaxed);
  } else if (c->hdr->magic != kMagic || c->hdr->version != kVersion) {
    munmap(p, size);
    close(fd);
    delete c;
    return nullptr;
  }
  return c;
}

void ring_doorbell(Page* pg, uint32_t gate, uint32_t old_gate) {
  if (gate != old_gate || gate) {
    pg->doorbell.fetch_add(1, std::memory_order_acq_rel);
    futex(&pg->doorbell, FUTEX_WAKE, 0x7fffffff, nullptr);
  }
}

// Second half of a deferred (torn) publish: the remaining fields, then the
// even sequence number.  Caller holds pub_mu.
void complete_torn(Page* pg, Ctl::Torn& t) {
  if (!t.active) return;
  pg->mask[1].store(t.mask1, std::memory_order_relaxed);
  pg->quantum_us.store(t.quantum, std::memory_order_relaxed);
  pg->priority.store(t.prio, std::memory_order_relaxed);
  pg->tenant_id.store(t.tid, std::memory_order_relaxed);
  pg->epoch.store(t.epoch, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  pg->seq.store(t.seq + 2, std::memory_order_release);
  t.active = false;
  ring_doorbell(pg, t.gate, t.old_gate);
}

// Seqlock publication of one page (caller holds pub_mu).  With `torn`, the
// publish stops half-written (odd sequence) and the bridge thread completes
// it after `torn_us` (the torn_page fault: readers must retry, never return
// a half-written assignment).
void publish_page(Page* pg, uint32_t gate, const uint64_t* mask, uint32_t quantum, int32_t prio, int32_t tid,
                  uint32_t epoch, Ctl::Torn* torn = nullptr, int64_t torn_us = -1) {
  if (torn) complete_torn(pg, *torn);  // a still-pending torn publish of this page lands first
  uint32_t s = pg->seq.load(std::memory_order_relaxed);
  const uint32_t old_gate = pg->gate.load(std::memory_order_relaxed);
  pg->seq.store(s + 1, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  pg->gate.store(gate, std::memory_order_relaxed);
  pg->mask[0].store(mask[0], std::memory_order_relaxed);
  if (torn && torn_us >= 0) {
    torn->active = true;
    torn->due = now_ns() + std::max<int64_t>(torn_us, 50) * 1000;
    torn->mask1 = mask[1];
    torn->quantum = quantum;
    torn->prio = prio;
    torn->tid = tid;
    torn->epoch = epoch;
    torn->seq = s;
    torn->gate = gate;
    torn->old_gate = old_gate;
    return;
  }
  pg->mask[1].store(mask[1], std::memory_order_relaxed);
  pg->quantum_us.store(quantum, std::memory_order_relaxed);
  pg->priority.store(prio, std::memory_order_relaxed);
  pg->tenant_id.store(tid, std::memory_order_relaxed);
  pg->epoch.store(epoch, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  pg->seq.store(s + 2, std::memory_order_release);
  ring_doorbell(pg, gate, old_gate);
}

// Complete every deferred publish that is due (all of them with force).
void complete_due_torn(Ctl* c, bool force) {
  std::lock_guard<std::mutex> g(c->pub_mu);
  const int64_t t = now_ns();
  for (size_t i = 0; i < c->torn.size(); ++i)
    if (c->torn[i].active && (force || t >= c->torn[i].due)) complete_torn(&c->pages[i], c->torn[i]);
}

// Seqlock reader back-off: spin briefly, then yield; a writer that died
// mid-publish (odd sequence forever) makes the read fail with -EAGAIN after
// ~50 ms instead of hanging the tenant at 100 % CPU.
struct SeqBackoff {
  int spins = 0;
  int64_t t0 = 0;
  bool again() {
    if (++spins < 64) {
      __builtin_ia32_pause();
      return true;
    }
    if (!t0) t0 = now_ns();
    if (now_ns() - t0 > 50000000) return false;
    sched_yield();
    return true;
  }
};

// ----------------------------------------------------------------- bridge --

void br_on_switch(void* user, int part, int prev, int next, int slot, int32_t q, int64_t now) {
  Ctl* c = (Ctl*)user;
  if (c->chained.on_switch) c->chained.on_switch(c->chained.user, part, prev, next, slot, q, now);
  if (part >= 128) return;
  const uint64_t bit = 1ull << (part & 63);
  const int w = part >> 6;
  if (prev >= 0 && prev < (int)c->pend_mask.size() / 2) c->pend_mask[2 * prev + w] &= ~bit;
  if (next >= 0 && next < (int)c->pend_mask.size() / 2) c->pend_mask[2 * next + w] |= bit;
}

void br_on_flush(void* user, int64_t now) {
  Ctl* c = (Ctl*)user;
  if (c->chained.on_flush) c->chained.on_flush(c->chained.user, now);
  std::lock_guard<std::mutex> g(c->pub_mu);
  c->epoch++;
  for (uint32_t i = 0; i < c->hdr->ntenants; ++i) {
    Page* pg = &c->pages[i];
    const int tid = pg->tenant_id.load(std::memory_order_relaxed);
    if (tid < 0 || tid >= (int)c->pend_mask.size() / 2) continue;
    // A torn publish of this page still pending (GPBS_FAULT torn_page) lands
    // first: the fields read below and the equality test must see the page
    // as it will be, not half-written (the deferred quantum was
    // otherwise overwritten with the stale value, and a mask equal to the
    // half-written one skipped its publish).
    if (c->torn[i].active) complete_torn(pg, c->torn[i]);
    const uint64_t m[2] = {c->pend_mask[2 * tid], c->pend_mask[2 * tid + 1]};
    if (m[0] == pg->mask[0].load(std::memory_order_relaxed) && m[1] == pg->mask[1].load(std::memory_order_relaxed)) continue;
    publish_page(pg, (m[0] | m[1]) ? 1u : 0u, m, pg->quantum_us.load(std::memory_order_relaxed),
                 pg->priority.load(std::memory_order_relaxed), tid, c->epoch, &c->torn[i],
                 gpbs_fault_fire(c->engine, "torn_page"));
  }
}

void br_on_park(void* user, int t, int s, int parked) {
  Ctl* c = (Ctl*)user;
  if (c->chained.on_park) c->chained.on_park(c->chained.user, t, s, parked);
}

// vPMU mirror publication (single writer: the bridge thread).
void publish_vpmu(Page* pg, const uint64_t* c4, uint64_t miss_rate, uint32_t tslice, int32_t cls, uint32_t phase) {
  const uint32_t s = pg->vseq.load(std::memory_order_relaxed);
  pg->vseq.store(s + 1, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  for (int k = 0; k < 4; ++k) pg->vpmu[k].store(c4[k], std::memory_order_relaxed);
  pg->vmiss_rate.store(miss_rate, std::memory_order_relaxed);
  pg->vtslice_us.store(tslice, std::memory_order_relaxed);
  pg->vclass.store(cls, std::memory_order_relaxed);
  pg->vphase.store(phase, std::memory_order_relaxed);
  pg->vseq.store(s + 2, std::memory_order_release);
}

void bridge_loop(Ctl* c) {
  std::vector<Report> buf(kRing);
  int64_t next_vpmu = 0;
  while (!c->stop.load(std::memory_order_acquire)) {
    // vPMU mirror every metric period (1 ms), not every 100 us poll: each
    // publication reads the tenant under the engine lock
    const bool vpmu_due = now_ns() >= next_vpmu;
    if (vpmu_due) next_vpmu = now_ns() + 1000000;
    for (uint32_t i = 0; i < c->hdr->ntenants; ++i) {
      Page* pg = &c->pages[i];
      const int tid = pg->tenant_id.load(std::memory_order_acquire);
      if (tid < 0) continue;
      // work state -> wake/block (vcpu_unblock / do_block)
      const uint32_t w = pg->has_work.load(std::memory_order_acquire);
      if (w != c->last_work[i]) {
        c->last_work[i] = w;
        if (w)
          gpbs_slot_wake(c->engine, tid, -1);
        else
          gpbs_slot_block(c->engine, tid, -1);
      }
      // reports -> vcrd_op
      uint32_t tail = pg->rtail.load(std::memory_order_relaxed);
      const uint32_t head = pg->rhead.load(std::memory_order_acquire);
      while (tail != head) {
        const Report r = pg->ring[tail % kRing];
        gpbs_report_wait(c->engine, tid, r.wait_ns, (int)r.kind);
        ++tail;
      }
      pg->rtail.store(tail, std::memory_order_release);
      // heartbeat
      const uint64_t hb = pg->heartbeat_ns.load(std::memory_order_acquire);
      if ((uint32_t)hb != c->last_hb_sent[i]) {
        c->last_hb_sent[i] = (uint32_t)hb;
        gpbs_tenant_heartbeat(c->engine, tid);
      }
      // tenant software counters -> slot 0 pmc (per-tenant sum is what PBS reads)
      uint64_t pmc[4];
      bool any = false;
      for (int k = 0; k < 4; ++k) {
        pmc[k] = pg->counters[k].load(std::memory_order_relaxed);
        any |= pmc[k] != 0;
      }
      if (any) {
        const int sid = gpbs_slot_id(c->engine, tid, 0);
        if (sid >= 0) gpbs_slot_set_pmc(c->engine, sid, pmc);
      }
      if (vpmu_due) {
        uint64_t tot[4];
        gpbs_tenant_info_t ti;
        if (gpbs_tenant_vpmu(c->engine, tid, tot) == 0 && gpbs_tenant_info(c->engine, tid, &ti) == 0)
          publish_vpmu(pg, tot, ti.cache_miss_rate, ti.tslice_us, gpbs_tenant_class(c->engine, tid), ti.phase);
      }
    }
    complete_due_torn(c, false);
    timespec ts{0, 100000};  // 100 us poll
    nanosleep(&ts, nullptr);
  }
  complete_due_torn(c, true);
}

}  // namespace

extern "C" {

void* gpbs_ctl_create(const char* name, int ntenants) {
  if (!name || ntenants <= 0 || ntenants > 4096) return nullptr;
  return map_region(name, ntenants, true);
}

void* gpbs_ctl_open(const char* name) {
  if (!name) return nullptr;
  return map_region(name, 0, false);
}

int gpbs_ctl_ntenants(void* h) { return h ? (int)((Ctl*)h)->hdr->ntenants : 0; }

void gpbs_ctl_close(void* h, int unlink_region) {
  Ctl* c = (Ctl*)h;
  if (!c) return;
  if (c->th.joinable()) {
    c->stop = true;
    c->th.join();
    gpbs_set_actuator_ops(c->engine, c->chained.on_switch || c->chained.on_flush ? &c->chained : nullptr);
  }
  munmap(c->hdr, c->size);
  close(c->fd);
  if (unlink_region) shm_unlink(c->name.c_str());
  delete c;
}

void gpbs_ctl_publish(void* h, int t, uint32_t gate, uint64_t mask, uint32_t quantum_us, int32_t prio, int32_t tid,
                      uint32_t epoch) {
  Page* pg = page(h, t);
  if (!pg) return;
  const uint64_t m[2] = {mask, 0};
  Ctl* c = (Ctl*)h;
  std::lock_guard<std::mutex> g(c->pub_mu);
  publish_page(pg, gate, m, quantum_us, prio, tid, epoch, (size_t)t < c->torn.size() ? &c->torn[t] : nullptr);
}

// Seqlock read; returns the number of retries (torn reads observed).
int gpbs_ctl_read(void* h, int t, uint32_t* gate, uint64_t* mask, uint32_t* quantum, int32_t* prio, int32_t* tid,
                  uint32_t* epoch) {
  Page* pg = page(h, t);
  if (!pg) return -22;
  int retries = 0;
  SeqBackoff bo;
  for (;;) {
    const uint32_t s0 = pg->seq.load(std::memory_order_acquire);
    if (s0 & 1) {
      ++retries;
      if (!bo.again()) return -11;
      continue;
    }
    const uint32_t g = pg->gate.load(std::memory_order_relaxed);
    const uint64_t m = pg->mask[0].load(std::memory_order_relaxed);
    const uint32_t q = pg->quantum_us.load(std::memory_order_relaxed);
    const int32_t p = pg->priority.load(std::memory_order_relaxed);
    const int32_t i = pg->tenant_id.load(std::memory_order_relaxed);
    const uint32_t e = pg->epoch.load(std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_acquire);
    if (pg->seq.load(std::memory_order_relaxed) == s0) {
      if (gate) *gate = g;
      if (mask) *mask = m;
      if (quantum) *quantum = q;
      if (prio) *prio = p;
      if (tid) *tid = i;
      if (epoch) *epoch = e;
      return retries;
    }
    ++retries;
    if (!bo.again()) return -11;
  }
}

int gpbs_ctl_read_vpmu(void* h, int t, uint64_t* c4, uint64_t* miss_rate, uint32_t* tslice_us, int32_t* cls,
                       uint32_t* phase, uint32_t* seq) {
  Page* pg = page(h, t);
  if (!pg) return -22;
  int retries = 0;
  SeqBackoff bo;
  for (;;) {
    const uint32_t s0 = pg->vseq.load(std::memory_order_acquire);
    if (s0 & 1) {
      ++retries;
      if (!bo.again()) return -11;
      continue;
    }
    uint64_t v[4];
    for (int k = 0; k < 4; ++k) v[k] = pg->vpmu[k].load(std::memory_order_relaxed);
    const uint64_t mr = pg->vmiss_rate.load(std::memory_order_relaxed);
    const uint32_t ts = pg->vtslice_us.load(std::memory_order_relaxed);
    const int32_t cl = pg->vclass.load(std::memory_order_relaxed);
    const uint32_t ph = pg->vphase.load(std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_acquire);
    if (pg->vseq.load(std::memory_order_relaxed) == s0) {
      if (c4)
        for (int k = 0; k < 4; ++k) c4[k] = v[k];
      if (miss_rate) *miss_rate = mr;
      if (tslice_us) *tslice_us = ts;
      if (cls) *cls = cl;
      if (phase) *phase = ph;
      if (seq) *seq = s0 / 2;
      return retries;
    }
    ++retries;
    if (!bo.again()) return -11;
  }
}

int gpbs_ctl_report(void* h, int t, uint64_t wait_ns, uint32_t kind, uint32_t gpu) {
  Page* pg = page(h, t);
  if (!pg) return -22;
  const uint32_t head = pg->rhead.load(std::memory_order_relaxed);
  const uint32_t tail = pg->rtail.load(std::memory_order_acquire);
  if (head - tail >= (uint32_t)kRing) {
    pg->dropped.fetch_add(1, std::memory_order_relaxed);
    return -28;
  }
  pg->ring[head % kRing] = Report{wait_ns, kind, gpu};
  pg->rhead.store(head + 1, std::memory_order_release);
  return 0;
}

int gpbs_ctl_drain(void* h, int t, uint64_t* waits, uint32_t* kinds, int max) {
  Page* pg = page(h, t);
  if (!pg) return -22;
  uint32_t tail = pg->rtail.load(std::memory_order_relaxed);
  const uint32_t head = pg->rhead.load(std::memory_order_acquire);
  int n = 0;
  while (tail != head && n < max) {
    const Report r = pg->ring[tail % kRing];
    if (waits) waits[n] = r.wait_ns;
    if (kinds) kinds[n] = r.kind;
    ++n;
    ++tail;
  }
  pg->rtail.store(tail, std::memory_order_release);
  return n;
}

void gpbs_ctl_heartbeat(void* h, int t, uint64_t now, uint32_t progress) {
  Page* pg = page(h, t);
  if (!pg) return;
  pg->heartbeat_ns.store(now ? now : (uint64_t)now_ns(), std::memory_order_release);
  pg->progress.store(progress, std::memory_order_relaxed);
  pg->pid.store((int32_t)getpid(), std::memory_order_relaxed);
}

int gpbs_ctl_status(void* h, int t, uint64_t* heartbeat, uint64_t* dropped, uint32_t* has_work, uint32_t* progress) {
  Page* pg = page(h, t);
  if (!pg) return -22;
  if (heartbeat) *heartbeat = pg->heartbeat_ns.load(std::memory_order_acquire);
  if (dropped) *dropped = pg->dropped.load(std::memory_order_relaxed);
  if (has_work) *has_work = pg->has_work.load(std::memory_order_acquire);
  if (progress) *progress = pg->progress.load(std::memory_order_relaxed);
  return pg->pid.load(std::memory_order_relaxed);
}

void gpbs_ctl_set_counters(void* h, int t, const uint64_t* c4) {
  Page* pg = page(h, t);
  if (!pg) return;
  for (int k = 0; k < 4; ++k) pg->counters[k].store(c4[k], std::memory_order_relaxed);
}

void gpbs_ctl_get_counters(void* h, int t, uint64_t* c4) {
  Page* pg = page(h, t);
  if (!pg) return;
  for (int k = 0; k < 4; ++k) c4[k] = pg->counters[k].load(std::memory_order_relaxed);
}

void gpbs_ctl_set_work(void* h, int t, int has_work) {
  Page* pg = page(h, t);
  if (pg) pg->has_work.store(has_work ? 1u : 0u, std::memory_order_release);
}

void gpbs_ctl_ring(void* h, int t) {
  Page* pg = page(h, t);
  if (!pg) return;
  pg->doorbell.fetch_add(1, std::memory_order_acq_rel);
  futex(&pg->doorbell, FUTEX_WAKE, 0x7fffffff, nullptr);
}

// Block until the doorbell changes (or timeout). Returns 1 on ring, 0 on timeout.
int gpbs_ctl_doorbell_wait(void* h, int t, int64_t timeout_ns) {
  Page* pg = page(h, t);
  if (!pg) return -22;
  const uint32_t v = pg->doorbell.load(std::memory_order_acquire);
  timespec ts{(time_t)(timeout_ns / 1000000000ll), (long)(timeout_ns % 1000000000ll)};
  futex(&pg->doorbell, FUTEX_WAIT, v, timeout_ns > 0 ? &ts : nullptr);
  return pg->doorbell.load(std::memory_order_acquire) != v ? 1 : 0;
}

// Full 128-partition assignment mask (8 GPUs x 8 XCDs x 2 halves) under the
// seqlock; returns the gate word.
int gpbs_ctl_read_mask(void* h, int t, uint64_t* mask2, uint32_t* epoch) {
  Page* pg = page(h, t);
  if (!pg) return -22;
  SeqBackoff bo;
  for (;;) {
    const uint32_t s0 = pg->seq.load(std::memory_order_acquire);
    if (s0 & 1) {
      if (!bo.again()) return -11;
      continue;
    }
    const uint32_t g = pg->gate.load(std::memory_order_relaxed);
    const uint64_t m0 = pg->mask[0].load(std::memory_order_relaxed), m1 = pg->mask[1].load(std::memory_order_relaxed);
    const uint32_t e = pg->epoch.load(std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_acquire);
    if (pg->seq.load(std::memory_order_relaxed) == s0) {
      if (mask2) {
        mask2[0] = m0;
        mask2[1] = m1;
      }
      if (epoch) *epoch = e;
      return (int)g;
    }
    if (!bo.again()) return -11;
  }
}

// Launch gate: wait until the scheduler lets the tenant launch. 1 open, 0 timeout.
int gpbs_ctl_wait_gate(void* h, int t, int64_t timeout_ns) {
  Page* pg = page(h, t);
  if (!pg) return -22;
  const int64_t deadline = now_ns() + timeout_ns;
  for (;;) {
    uint32_t gate = 0;
    gpbs_ctl_read(h, t, &gate, nullptr, nullptr, nullptr, nullptr, nullptr);
    if (gate) return 1;
    const int64_t left = deadline - now_ns();
    if (timeout_ns > 0 && left <= 0) return 0;
    gpbs_ctl_doorbell_wait(h, t, timeout_ns > 0 ? std::min<int64_t>(left, 1000000) : 1000000);
  }
}

// Bind a region to an engine: page i serves engine tenant pages[i].tenant_id.
int gpbs_ctl_bind(void* h, void* engine) {
  Ctl* c = (Ctl*)h;
  if (!c || !engine || c->th.joinable()) return -22;
  c->engine = (gpbs_engine_t*)engine;
  c->pend_mask.assign(2 * 4096, 0);
  c->last_work.assign(c->hdr->ntenants, 0);
  c->last_hb_sent.assign(c->hdr->ntenants, 0);
  {
    std::lock_guard<std::mutex> g(c->pub_mu);
    c->torn.assign(c->hdr->ntenants, Ctl::Torn{});
  }
  gpbs_actuator_ops_t a{};
  a.user = c;
  a.on_switch = br_on_switch;
  a.on_flush = br_on_flush;
  a.on_park = br_on_park;
  c->chained = gpbs_actuator_ops_t{};
  gpbs_get_actuator_ops(c->engine, &c->chained);
  gpbs_set_actuator_ops(c->engine, &a);
  c->stop = false;
  c->th = std::thread(bridge_loop, c);
  return 0;
}

// Register engine tenant `tid` on page t (daemon side).
int gpbs_ctl_assign(void* h, int t, int tid) {
  Page* pg = page(h, t);
  if (!pg) return -22;
  const uint64_t m[2] = {0, 0};
  Ctl* c = (Ctl*)h;
  std::lock_guard<std::mutex> g(c->pub_mu);
  if (pg->tenant_id.load(std::memory_order_acquire) < 0) {  // the bridge skips unassigned pages: no second writer
    const uint64_t z[4] = {0, 0, 0, 0};
    publish_vpmu(pg, z, 0, 0, -1, 0);
  }
  publish_page(pg, 0, m, 0, 0, tid, 0, (size_t)t < c->torn.size() ? &c->torn[t] : nullptr);
  return 0;
}

}  // extern "C"
