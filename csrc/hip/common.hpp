// Shared definitions for the gfx950 (MI355X / CDNA4) kernels and runtime.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

namespace gpbs_hip {

constexpr int kXcds = 8;          // MI355X: 8 XCDs x 32 CUs
constexpr int kMaxTenants = 64;   // per GPU context
constexpr int kNumPmc = 4;        // INST, CYCLES, L2_REFS, L2_MISSES (modeled)
constexpr uint32_t kNoOwner = 0xFFFFFFFFu;
// Bit 31 of an owner word: XCD split into CU halves (spatial mode, set on both
// words of the XCD when its two owners are of different contention classes).
constexpr uint32_t kSplitBit = 0x80000000u;
constexpr uint32_t kOwnerMask = 0x7FFFFFFFu;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16;
typedef unsigned int u32;
typedef unsigned long long u64;

// Partition table shared by the scheduler (host) and tenant kernels.  Lives
// in fine-grained pinned host memory: the dispatcher thread's store is seen
// by the next system-scope load of a workgroup (~1-2 us over PCIe) without a
// copy or a kernel launch.  A device-memory copy is maintained by the
// partition_switch kernel when GPBS_TABLE=device.
// Each XCD exposes up to kCtx issue contexts (the SMT-sibling analog: the
// tenants' waves co-reside on the XCD's CUs, typically one MFMA-bound and
// the others memory-bound).  owner[kCtx*x + c] is the tenant running on
// context c of XCD x; an engine uses nctx <= kCtx of them, the rest stay
// kNoOwner.
constexpr int kCtx = 4;
struct alignas(64) PartTable {
  u32 epoch;
  u32 flags;
  u32 hold;     // latency request in flight: GATE_HOLD tenants pause at their next unit (host-written)
  u32 pad0;
  union {
    u32 owner[kXcds * kCtx];  // tenant id per (XCD, context), kNoOwner when idle
    u64 pair[kXcds][2];       // contexts {0,1} and {2,3} of an XCD, 8 bytes each
  };
  u32 pad[12];
};
static_assert(sizeof(PartTable) == 192, "partition table layout");

// Work queue of one tenant kernel invocation (tile / chunk queue).
struct alignas(64) WorkQueue {
  u32 next;       // next unit to grab (atomic); XCD-range queues: units claimed
  u32 done;       // completed units
  u32 exited;     // workgroups that finished (any path)
  u32 stopped;    // workgroups that left because their XCD was revoked
  u32 xnext[kXcds];  // XCD-range queues: next offset within range x
  u32 pad[4];
};

// Exit protocol of every tenant kernel: the last workgroup to leave publishes
// the unit count to the host-visible status word (pinned, system scope), so the
// runner learns "finished or revoked" from the completion event alone.
// Last workgroup out reports the unit and resets the queue.  No agent-scope
// fence: on a
// multi-XCD gfx950 an agent-scope release writes back the XCD's whole L2, so
// 256 workgroups each fencing after storing their C tiles pay for the dirty
// lines of everyone's output; ordering is all the protocol needs -- every
// done increment must be performed before the same workgroup's exited
// increment -- and a vmcnt(0) wait (atomics count in vmcnt on gfx9) gives
// exactly that.  Kernel completion still releases C to the host / next
// kernel.  Measured on the 4096^3 GEMM: 1153 vs 1094 TF/s with the fences
// (scripts/kbench.py, profiles/r3/kbench_gemm_h.log).
__device__ __forceinline__ void finish(WorkQueue* q, u32* status, u32 total) {
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const u32 old = atomicAdd(&q->exited, 1u);
    if (old == gridDim.x - 1) {
      const u32 d = __hip_atomic_load(&q->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (status) __hip_atomic_store(status, d | 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      // the exit bookkeeping is reset by the last workgroup out in both
      // cases -- a revoked unit's relaunch needs no fill kernel on the
      // tenant's queue (round 6: 1443 fillBufferAligned per 8mix run before)
      __hip_atomic_store(&q->exited, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&q->stopped, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d >= total) {
        __hip_atomic_store(&q->next, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&q->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int x = 0; x < kXcds; ++x) __hip_atomic_store(&q->xnext[x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}


// Gate modes passed to tenant kernels.
// GATE_NONE: run anywhere; GATE_TABLE: leave revoked XCDs; GATE_PARK: sleep
// on revoked XCDs (bounded) and resume when the XCD is handed back.
// Bit 2 (GATE_DEVTABLE): the table is the device-memory copy refreshed by
// k_partition_switch (agent-scope polls served on chip) instead of the
// pinned host table (system-scope polls over PCIe).
// Bit 3 (GATE_SPATIAL): the two partitions of an XCD are CU halves (shader
// engines 0-1 vs 2-3) instead of co-resident issue contexts; a workgroup
// checks only the entry of the half its CU belongs to.
enum GateMode : u32 {
  GATE_NONE = 0, GATE_TABLE = 1, GATE_PARK = 2, GATE_DEVTABLE = 4, GATE_SPATIAL = 8,
  GATE_WAVEPRIO = 16,  // latency-class tenant: its waves win SIMD issue arbitration (s_setprio 3)
  // Bit 5 (GATE_SE): the four partitions of an XCD are its four shader
  // engines (8 CUs each), owned EXCLUSIVELY: a workgroup runs only on the SE
  // whose owner word names its tenant.  Exclusive SE ownership is what makes
  // the SE-resolved SQ/TCP hardware counters attributable per tenant
  // (profiles/hwc/se_separation_probe.txt).
  GATE_SE = 32,
  // Bit 6 (GATE_HOLD): before grabbing a unit, wait (bounded) while the
  // table's hold word is set -- the latency tenant's request is in flight.
  // Given to memory-class tenants only: the request (a GEMV) is HBM-bound, and
  // their next chunk boundary comes within ~25 us.  The wake-BOOST of
  // X:xen/common/sched_credit.c:1080-1084 for an I/O-bound domain, as a pause
  // of the tenants that contend with it instead of a preemption of all.
  GATE_HOLD = 64,
};
constexpr u32 kParkSpins = 100;  // x ~20 us
constexpr u32 kHoldSpins = 256;  // x ~0.9 us: a stuck hold word costs at most ~0.25 ms per unit

#define HIPCHECK(x)                                                                              \
  do {                                                                                           \
    hipError_t _e = (x);                                                                         \
    if (_e != hipSuccess) {                                                                      \
      fprintf(stderr, "[gpbs-hip] %s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(_e)); \
      return -(int)_e - 1000;                                                                    \
    }                                                                                            \
  } while (0)

__device__ __forceinline__ u32 xcc_id() {
  // s_getreg_b32 hwreg(HW_REG_XCC_ID, 0, 4): the XCD this wave runs on.
  return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
}

__device__ __forceinline__ u32 hw_id() { return __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4); }

// CU half of this wave: HW_ID.SE_ID is bits 15:13; MI355X XCDs have four
// shader engines (logical CU i of an XCD sits on SE i % 4, measured with the
// census kernel under one-bit CU masks), so SE >> 1 splits an XCD 16/16.
__device__ __forceinline__ u32 cu_half() { return (hw_id() >> 14) & 1u; }

// Shader engine of this wave within its XCD (HW_ID.SE_ID bits 14:13; 0..3).
__device__ __forceinline__ u32 se_id() { return (hw_id() >> 13) & 3u; }

__device__ __forceinline__ u32 load_sys(const u32* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// GATE_HOLD (thread 0, before a unit grab): bounded wait while the hold word
// is set.  The word lives in the table the kernel was given: the pinned host
// table or the BAR-written VRAM table (the host raises and clears it); the
// kernel-refreshed device table never carries it.
__device__ __forceinline__ void hold_wait(const PartTable* t, u32 mode) {
  if (!(mode & GATE_HOLD)) return;
  for (u32 k = 0; k < kHoldSpins; ++k) {
    const u32 h = (mode & GATE_DEVTABLE) ? __hip_atomic_load(&t->hold, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                         : __hip_atomic_load(&t->hold, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (!h) return;
    __builtin_amdgcn_s_sleep(32);
  }
}

// Does tenant `me` own the XCD this workgroup runs on?
__device__ __forceinline__ bool owns(const PartTable* t, u32 mode, u32 me, u32 xcc) {
  if ((mode & 3) == GATE_NONE) return true;
  if (mode & GATE_SE) {
    const u32 se = se_id();
    const u32* w = t->owner + kCtx * (xcc & 7) + se;
    const u32 o = (mode & GATE_DEVTABLE) ? __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                         : __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return (o & kOwnerMask) == me;
  }
  // Two 8-byte loads (one cache line) cover the four contexts of the XCD.
  const u64* q = t->pair[xcc & 7];
  const u64 p01 = (mode & GATE_DEVTABLE) ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                         : __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const u32 w0 = (u32)p01, w1 = (u32)(p01 >> 32);
  const bool h0 = (w0 & kOwnerMask) == me, h1 = (w1 & kOwnerMask) == me;
  if (!(mode & GATE_SPATIAL) || (h0 && h1)) {
    if (h0 || h1) return true;
    const u64 p23 = (mode & GATE_DEVTABLE) ? __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                           : __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return (u32)p23 == me || (u32)(p23 >> 32) == me;
  }
  // Spatial (contexts 0/1 only): a split XCD confines each owner to its CU
  // half; an unsplit one (same-class owners, or the other side idle) is
  // shared in full.
  if (h0) return !(w0 & kSplitBit) || cu_half() == 0;
  if (h1) return !(w1 & kSplitBit) || cu_half() == 1;
  return false;
}

// Per-(tenant, xcd) software counter block, accumulated at workgroup exit.
// System-scope atomics: the block lives in fine-grained VRAM that the host
// sampler reads through the BAR every metric tick (csrc/hip/runtime.cpp
// read_block), so each add is performed past the XCD's L2, where the host's
// read sees it.
__device__ __forceinline__ void count(u64* cnt, u32 me, u32 xcc, u64 inst, u64 cyc, u64 refs, u64 miss) {
  if (!cnt) return;
  u64* c = cnt + ((size_t)me * kXcds + (xcc & 7)) * kNumPmc;
  if (inst) __hip_atomic_fetch_add(c + 0, inst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (cyc) __hip_atomic_fetch_add(c + 1, cyc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (refs) __hip_atomic_fetch_add(c + 2, refs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (miss) __hip_atomic_fetch_add(c + 3, miss, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Work-queue unit grab of a persistent tenant workgroup (thread 0 decides,
// workgroup-uniform): while its tenant owns the partition this workgroup runs
// on, the next unit index; -1 when the queue is drained or the partition was
// revoked (GATE_PARK: sleep there, bounded, and resume if handed back).
__device__ __forceinline__ int grab_unit(WorkQueue* q, const PartTable* table, u32 mode, u32 me, u32 xcc,
                                         int* s_slot, u32 total) {
  if (threadIdx.x == 0) {
    int u = -1;
    hold_wait(table, mode);
    for (u32 spins = 0;; ++spins) {
      if (owns(table, mode, me, xcc)) {
        const u32 t = atomicAdd(&q->next, 1u);
        u = t < total ? (int)t : -1;
        break;
      }
      // GATE_PARK: stay resident (sleeping) on a revoked XCD so the workgroup
      // resumes within ~20 us when the scheduler hands the XCD back, instead
      // of waiting for the next launch.  Bounded (~2 ms): a workgroup that is
      // not rescheduled leaves and the runner relaunches the rest of the unit.
      if ((mode & 3) != GATE_PARK || spins >= kParkSpins ||
          __hip_atomic_load(&q->next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= total) {
        atomicAdd(&q->stopped, 1u);
        break;
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) __builtin_amdgcn_s_sleep(127);
    }
    *s_slot = u;
  }
  __syncthreads();
  int u = *s_slot;
  __syncthreads();
  return u;
}

// XCD-range variant: units are split into 8 contiguous ranges and a
// workgroup first drains the range of the XCD it runs on, then steals from
// the others in ring order.  Neighbouring tiles (which share operand panels)
// thus meet in one XCD's private L2 -- the XCD-aware blockIdx remap of a plain
// grid, done on a work queue so gating, parking and relaunch still hold.

// Per-unit counter accounting (modeled per-tile counters) + done count.
__device__ __forceinline__ void count_unit(u64* cnt, u32 me, u32 xcc, u64 inst, u64* t_last, u64 refs, u64 miss,
                                           WorkQueue* q) {
  if (threadIdx.x != 0) return;
  const u64 t = __builtin_amdgcn_s_memtime();
  count(cnt, me, xcc, inst, t - *t_last, refs, miss);
  *t_last = t;
  atomicAdd(&q->done, 1u);
}

}  // namespace gpbs_hip
