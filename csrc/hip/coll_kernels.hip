// All-reduce tenant over xGMI with IPC-mapped peer buffers (N > 1 GPUs of one
// node, one process per GPU): the interference generator of BASELINE config
// #3/#4 written as a gpbs tenant kernel, so -- unlike RCCL's kernels -- it is
// confined by the partition table like every other tenant (GATE_SE per
// workgroup, CU-masked class-half streams) and its traffic is attributable
// to it by shader-engine ownership.
//
// One unit = one all-reduce of the rank's input buffer, direct (one-shot
// reduce-scatter + all-gather over the fully connected xGMI mesh: every
// MI355X links to each of its 7 peers):
//   * rank r owns slice r of the vector (n8 / world 16-byte vectors); its
//     workgroups grab chunks of the slice from the work queue, load the chunk
//     from all `world` peers' inputs (xGMI reads), sum in fp32, and store the
//     bf16 result into all peers' outputs (xGMI writes);
//   * units are collective: unit `seq` starts only after every peer finished
//     unit seq-1 -- a P2P-flag barrier in device memory: each rank's last
//     workgroup out stores seq+1 into its word of every peer's flag array
//     (system-scope store over xGMI), and the first thing a workgroup does is
//     wait for all of its own flag words to reach seq.  A rank whose tenant is
//     descheduled stalls its peers -- the symptom gang scheduling removes
//     (C16), measured by the engine's K10 wait reports.
// A workgroup that waits while its shader engine is revoked leaves (the
// runner relaunches the unit later).  So does one that has waited
// yield_ticks: a kernel spinning on a peer must not hold the GPU, since when
// ranks share a device (tests: 2 processes on one GPU) the hardware
// scheduler time-slices their queues and a resident spinning grid can keep
// the peer's kernel from ever being dispatched (measured: both ranks stuck
// until the timeout).  Every wait is bounded by the wall clock, so a dead
// peer ends the kernel with an error bit instead of a hang; the runner
// bounds a unit's relaunches by the same timeout.
#include "common.hpp"

namespace gpbs_hip {

constexpr int kCollMax = 8;

struct CollDesc {
  const u32x4* in[kCollMax];  // rank q's input (bf16 x 8 per vector), mapped into this process
  u32x4* out[kCollMax];       // rank q's output
  u32* flags[kCollMax];       // rank q's flag words [kCollMax] (word s: units rank s has finished)
  u32 rank, world;
  u64 n8;                     // 16-byte vectors per buffer
};

constexpr u32 kCollErrBit = 0x40000000u;  // status bit: a peer barrier timed out

__device__ __forceinline__ float bflo(u32 w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfhi(u32 w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ u32 f2bf_rne(float f) {
  const u32 u = __float_as_uint(f);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

constexpr int CNT = 256, CU_ = 4;

__global__ __launch_bounds__(CNT) void k_allreduce(const CollDesc* __restrict__ d, u32 seq, u32 chunk8, WorkQueue* q,
                                                   const PartTable* table, u32 mode, u32 me, u64* cnt, u32* status,
                                                   u64 timeout_ticks, u64 yield_ticks) {
  __shared__ int s_slot[4];
  __shared__ int s_ok;
  const u32 xcc = xcc_id();
  const u32 rank = d->rank, world = d->world;
  const u64 per = (d->n8 + world - 1) / world;
  const u64 lo = (u64)rank * per, hi = min(lo + per, d->n8);
  const u32 nchunks = hi > lo ? (u32)((hi - lo + chunk8 - 1) / chunk8) : 0u;
  // 1. collective barrier: every peer has finished unit seq - 1
  if (threadIdx.x == 0) {
    int ok = 1;
    const u64 t0 = wall_clock64();
    const u32* fl = d->flags[rank];
    for (;;) {
      bool all = true;
      for (u32 s = 0; s < world; ++s)
        if (__hip_atomic_load(fl + s, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) all = false;
      if (all) break;
      if (!owns(table, mode, me, xcc)) {
        ok = 0;  // revoked while waiting: leave, the runner relaunches the unit
        break;
      }
      const u64 el = wall_clock64() - t0;
      if (el > timeout_ticks) {
        ok = -1;
        break;
      }
      if (el > yield_ticks) {
        ok = 0;  // give the GPU back; the runner relaunches the unit
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
    s_ok = ok;
  }
  __syncthreads();
  const int ok = s_ok;
  u64 t_last = __builtin_amdgcn_s_memtime();
  const u64 lines = (u64)chunk8 * 16 / 128;
  const u64 inst = (u64)chunk8 * (world + world) / 64 + (u64)chunk8 * 16 / 64;
  if (ok > 0) {
    for (;;) {
      const int c = grab_unit(q, table, mode, me, xcc, s_slot, nchunks);
      if (c < 0) break;
      const u64 base = lo + (u64)c * chunk8, end = min(base + chunk8, hi);
      for (u64 i = base + threadIdx.x; i < end; i += (u64)CNT * CU_) {
        float acc[CU_][8];
#pragma unroll
        for (int k = 0; k < CU_; ++k)
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
        for (u32 s = 0; s < world; ++s) {
          u32x4 v[CU_];
#pragma unroll
          for (int k = 0; k < CU_; ++k) {
            const u64 idx = i + (u64)k * CNT;
            if (idx < end) v[k] = __builtin_nontemporal_load(d->in[s] + idx);
          }
#pragma unroll
          for (int k = 0; k < CU_; ++k)
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              acc[k][2 * w] += bflo(v[k][w]);
              acc[k][2 * w + 1] += bfhi(v[k][w]);
            }
        }
#pragma unroll
        for (int k = 0; k < CU_; ++k) {
          const u64 idx = i + (u64)k * CNT;
          if (idx >= end) continue;
          u32x4 r;
#pragma unroll
          for (int w = 0; w < 4; ++w) r[w] = f2bf_rne(acc[k][2 * w]) | (f2bf_rne(acc[k][2 * w + 1]) << 16);
          for (u32 s = 0; s < world; ++s) __builtin_nontemporal_store(r, d->out[s] + idx);
        }
      }
      count_unit(cnt, me, xcc, inst, &t_last, (u64)(world + world) * lines, (u64)(world + world) * lines, q);
    }
  } else if (threadIdx.x == 0) {
    atomicAdd(&q->stopped, 1u);
    if (ok < 0) atomicOr(&q->pad[0], 1u);  // timed-out barrier: reported through the status word
  }
  // 2. exit: the last workgroup of a completed unit tells every peer
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: this WG's peer stores are visible
    const u32 old = atomicAdd(&q->exited, 1u);
    if (old == gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const u32 dn = __hip_atomic_load(&q->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const u32 err = __hip_atomic_load(&q->pad[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? kCollErrBit : 0u;
      if (dn >= nchunks && !err)
        for (u32 s = 0; s < world; ++s)
          __hip_atomic_store(d->flags[s] + rank, seq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (status) __hip_atomic_store(status, dn | err | 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      q->exited = 0;  // exit bookkeeping: reset for any relaunch (no fill kernel on the queue)
      q->stopped = 0;
      if (dn >= nchunks || err) {  // zero the queue for the next launch
        q->next = 0;
        q->done = 0;
        q->pad[0] = 0;
      }
      __threadfence();
    }
  }
}

// ---- gang epoch exchange over xGMI (the scheduler's cross-GPU
// barrier on the device, next to the host shm transport) -------------------
// Every rank owns a board in uncached device memory, IPC-mapped by every
// peer: [2 parities][world][stride] int64 words, slot r = rank r's entry
// (word 0: the exchange's sequence number, words 1..nvals: its values).  One
// exchange (one 64-lane wave): write this rank's values into its slot of
// EVERY peer's board, then its sequence number with a system-scope release;
// wait until every slot of its own board carries the sequence; copy the rows
// to the caller's pinned buffer.  Two parities: a rank starts exchange k+1
// only after finishing k, which needs every peer's write of k, which each
// peer makes only after finishing k-1 -- so k+1 never overwrites a slot
// someone still reads for k-1... and k+2 (same parity as k) is written only
// after every peer finished k.  A wait longer than yield_ticks leaves with
// status 1 and the host relaunches (a spinning grid must not hold a GPU it
// may share with a peer's queues; the lesson of k_allreduce).
struct GangDesc {
  long long* board[kCollMax];  // rank q's board, mapped into this process
  u32 rank, world, stride, nvals;
};

__global__ __launch_bounds__(64) void k_gang_exchange(const GangDesc* __restrict__ d, u32 seq,
                                                       const long long* __restrict__ vals, long long* out,
                                                       u32* status, u64 yield_ticks) {
  const u32 rank = d->rank, world = d->world, stride = d->stride, nv = d->nvals;
  const u32 par = seq & 1u;
  const size_t slot = ((size_t)par * world + rank) * stride;
  // 1. publish: values, then the sequence number, into every peer's board
  for (u32 s = 0; s < world; ++s)
    for (u32 t = threadIdx.x; t < nv; t += 64)
      __hip_atomic_store(d->board[s] + slot + 1 + t, vals[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the values before the sequence numbers
  __syncthreads();                                 // ... every lane's values, not just its own
  if (threadIdx.x < world)
    __hip_atomic_store(d->board[threadIdx.x] + slot, (long long)seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  // 2. wait for every rank's entry on this rank's board
  long long* mine = d->board[rank] + (size_t)par * world * stride;
  int ok = 1;
  if (threadIdx.x == 0) {
    const u64 t0 = wall_clock64();
    for (;;) {
      bool all = true;
      for (u32 r = 0; r < world; ++r)
        if (__hip_atomic_load(mine + (size_t)r * stride, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < (long long)seq)
          all = false;
      if (all) break;
      if (wall_clock64() - t0 > yield_ticks) {
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  ok = __shfl(ok, 0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  if (!ok) {
    if (threadIdx.x == 0) __hip_atomic_store(status, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  // 3. every rank's row to the caller
  for (u32 r = 0; r < world; ++r)
    for (u32 t = threadIdx.x; t < nv; t += 64)
      out[(size_t)r * nv + t] =
          __hip_atomic_load(mine + (size_t)r * stride + 1 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (threadIdx.x == 0) __hip_atomic_store(status, 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace gpbs_hip

using namespace gpbs_hip;

extern "C" {

int gpbs_hip_coll_desc_size(void) { return (int)sizeof(CollDesc); }
int gpbs_hip_gang_desc_size(void) { return (int)sizeof(GangDesc); }

int gpbs_hip_gang_exchange(const void* desc, unsigned seq, const void* vals, void* out, void* status,
                           unsigned long long yield_ticks, hipStream_t s) {
  hipLaunchKernelGGL(k_gang_exchange, dim3(1), dim3(64), 0, s, (const GangDesc*)desc, seq, (const long long*)vals,
                     (long long*)out, (u32*)status, (u64)yield_ticks);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// desc: device CollDesc; bytes: per-buffer size (multiple of 16 * world);
// seq: the unit's collective sequence number (0, 1, ...).
int gpbs_hip_allreduce(const void* desc, unsigned seq, unsigned long long bytes, unsigned chunk_bytes, void* q,
                       const void* table, unsigned mode, unsigned me, void* cnt, void* status, int grid,
                       unsigned long long timeout_ticks, unsigned long long yield_ticks, hipStream_t s) {
  if (bytes % 16 || chunk_bytes % 16 || chunk_bytes == 0) return -22;
  if (grid <= 0) grid = 256;
  if (yield_ticks == 0 || yield_ticks > timeout_ticks) yield_ticks = timeout_ticks;
  hipLaunchKernelGGL(k_allreduce, dim3(grid), dim3(CNT), 0, s, (const CollDesc*)desc, seq, chunk_bytes / 16,
                     (WorkQueue*)q, (const PartTable*)table, mode, me, (u64*)cnt, (u32*)status, (u64)timeout_ticks,
                     (u64)yield_ticks);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // extern "C"
