// Per-engine lock-free trace ring (xentrace analog: X:xen/common/trace.c:665-681,
// event classes X:xen/include/public/trace.h:56-86).  Fixed 32-byte records;
// a single producer (the engine, under its lock) and any number of readers
// that copy out by sequence number (lost records are reported, not blocked on).
#pragma once
#include <atomic>
#include <cstdint>
#include <vector>

namespace gpbs {

enum TraceEvent : uint32_t {
  TRC_SWITCH = 1,      // a0=partition a1=prev tenant a2=next tenant a3=quantum_us
  TRC_WAKE = 2,        // a0=tenant a1=slot a2=partition
  TRC_SLEEP = 3,       // a0=tenant a1=slot a2=partition
  TRC_ACCT = 4,        // a0=pool a1=weight_total a2=credit_total a3=balance
  TRC_ADAPT = 5,       // a0=tenant a1=old_us a2=new_us a3=(phase<<24)|err&0xffffff
  TRC_GANG_EPOCH = 6,  // a0=epoch a1=rank a2=ranks a3=latency_us
  TRC_REPORT = 7,      // a0=tenant a1=kind a2=wait_lo a3=wait_hi
  TRC_MIGRATE = 8,     // a0=tenant a1=slot a2=from a3=to
  TRC_PARK = 9,        // a0=tenant a1=slot a2=parked(1)/unparked(0)
  TRC_STEAL = 10,      // a0=tenant a1=slot a2=from a3=to
  TRC_METRIC = 11,     // a0=tenant a1=inst_lo a2=miss_lo a3=curr_rate
  TRC_DEAD = 12,       // a0=tenant (heartbeat lost)
  TRC_POOL = 13,       // a0=pool a1=op a2=arg
  TRC_FAULT = 14,      // a0=fault kind a1=arg
  TRC_ATC = 15,        // a0=global min slice a1=ntenants
  TRC_CLASS = 16,      // a0=tenant a1=class (0 compute, 1 memory) a2=partitions allowed
  TRC_GANG_TIMEOUT = 17,  // a0=epoch a1=rank a2=waited_us: gang deadline missed, rank degraded to local
};

struct TraceRecord {
  uint64_t t_ns;
  uint32_t event;
  uint32_t cpu;  // partition / rank that emitted it
  uint32_t a[4];
};
static_assert(sizeof(TraceRecord) == 32, "trace record is 32 bytes");

class TraceRing {
 public:
  explicit TraceRing(size_t capacity_pow2 = 1u << 16) : buf_(capacity_pow2), mask_(capacity_pow2 - 1) {}
  void set_mask(uint64_t event_mask) { evt_mask_.store(event_mask, std::memory_order_relaxed); }
  uint64_t event_mask() const { return evt_mask_.load(std::memory_order_relaxed); }
  void emit(uint64_t t, uint32_t ev, uint32_t cpu, uint32_t a0 = 0, uint32_t a1 = 0, uint32_t a2 = 0,
            uint32_t a3 = 0) {
    if (!(evt_mask_.load(std::memory_order_relaxed) & (1ull << ev))) return;
    uint64_t h = head_.load(std::memory_order_relaxed);
    TraceRecord& r = buf_[h & mask_];
    r.t_ns = t;
    r.event = ev;
    r.cpu = cpu;
    r.a[0] = a0;
    r.a[1] = a1;
    r.a[2] = a2;
    r.a[3] = a3;
    head_.store(h + 1, std::memory_order_release);
  }
  // Copy records with sequence >= *cursor (at most max). Advances *cursor;
  // returns count and sets *lost to records overwritten before being read.
  size_t read(uint64_t* cursor, TraceRecord* out, size_t max, uint64_t* lost) const {
    uint64_t h = head_.load(std::memory_order_acquire);
    uint64_t c = *cursor;
    uint64_t oldest = h > buf_.size() ? h - buf_.size() : 0;
    *lost = 0;
    if (c < oldest) {
      *lost = oldest - c;
      c = oldest;
    }
    size_t n = 0;
    while (c < h && n < max) out[n++] = buf_[(c++) & mask_];
    *cursor = c;
    return n;
  }
  uint64_t head() const { return head_.load(std::memory_order_acquire); }

 private:
  std::vector<TraceRecord> buf_;
  uint64_t mask_;
  std::atomic<uint64_t> head_{0};
  std::atomic<uint64_t> evt_mask_{~0ull};
};

}  // namespace gpbs
