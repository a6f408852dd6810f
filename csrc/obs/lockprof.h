// Lock profiling (the lock_profile=y / xenlockprof analog:
// X:xen/common/spinlock.c:88-115 keeps lock_cnt, block_cnt, time_hold and
// time_block per lock; X:tools/misc/xenlockprof.c prints them).  gpbs has one
// hot lock, the engine mutex, taken by the dispatcher thread and by every C
// ABI entry (tenant runners, RPC server, gang thread).  Counting is lock-free
// (relaxed atomics); only the outermost acquisition of the recursive lock is
// accounted.
#pragma once
#include <atomic>
#include <chrono>
#include <cstdint>

namespace gpbs {

struct LockProfile {
  std::atomic<uint64_t> lock_cnt{0};       // acquisitions
  std::atomic<uint64_t> block_cnt{0};      // acquisitions that found the lock held
  std::atomic<uint64_t> time_block_ns{0};  // total time spent waiting
  std::atomic<uint64_t> time_hold_ns{0};   // total time held
  std::atomic<uint64_t> max_block_ns{0};
  std::atomic<uint64_t> max_hold_ns{0};
  std::atomic<uint64_t> handoffs{0};       // dispatcher yielded the lock while behind schedule

  static uint64_t clock_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  static void bump_max(std::atomic<uint64_t>& m, uint64_t v) {
    uint64_t cur = m.load(std::memory_order_relaxed);
    while (v > cur && !m.compare_exchange_weak(cur, v, std::memory_order_relaxed)) {
    }
  }
  void acquired(bool blocked, uint64_t wait_ns) {
    lock_cnt.fetch_add(1, std::memory_order_relaxed);
    if (blocked) {
      block_cnt.fetch_add(1, std::memory_order_relaxed);
      time_block_ns.fetch_add(wait_ns, std::memory_order_relaxed);
      bump_max(max_block_ns, wait_ns);
    }
  }
  void released(uint64_t hold_ns) {
    time_hold_ns.fetch_add(hold_ns, std::memory_order_relaxed);
    bump_max(max_hold_ns, hold_ns);
  }
  void reset() {
    for (auto* a : {&lock_cnt, &block_cnt, &time_block_ns, &time_hold_ns, &max_block_ns, &max_hold_ns, &handoffs})
      a->store(0, std::memory_order_relaxed);
  }
};

}  // namespace gpbs
