// Tenant workload kernels for gfx950 (MI355X), partition-aware.
//
// Every kernel is a persistent grid over a WorkQueue: workgroups read their
// XCD id (HW_REG_XCC_ID), leave at once when the scheduler's partition table
// does not give that XCD to their tenant, and otherwise pull tiles/chunks with
// one atomic per unit, re-checking ownership between units.  This is the
// MI355X actuation of the reference's context switch: the credit scheduler
// hands XCD partitions to tenants and a revoked XCD drains within one tile
// (X:xen/arch/x86/domain.c:1584-1660 is what it replaces).  Each workgroup
// adds its modeled counters (instructions, busy cycles, L2 line references,
// HBM line fills) into a per-(tenant, XCD) block at exit: the vPMU analog
// (X:xen/arch/x86/perfctr.c:1547-1572).
#include "common.hpp"

namespace gpbs_hip {

// ---------------------------------------------------------------- helpers --

// Thread 0 decides for the whole workgroup: grab the next unit, or stop when
// the XCD was revoked.  Returns the unit index, or -1 to stop.
__device__ __forceinline__ int grab_unit(WorkQueue* q, const PartTable* table, u32 mode, u32 me, u32 xcc,
                                         int* s_slot, u32 total) {
  if (threadIdx.x == 0) {
    int u = -1;
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

// Per-unit counter accumulation by thread 0 (tile-granular vPMU: the scheduler
// sees a smooth rate instead of bursts at kernel exit).
__device__ __forceinline__ void count_unit(u64* cnt, u32 me, u32 xcc, u64 inst, u64* t_last, u64 refs, u64 miss,
                                           WorkQueue* q) {
  if (threadIdx.x != 0) return;
  const u64 t = __builtin_amdgcn_s_memtime();
  count(cnt, me, xcc, inst, t - *t_last, refs, miss);
  *t_last = t;
  atomicAdd(&q->done, 1u);
}

__device__ __forceinline__ u16 f2bf(float x) { return __builtin_bit_cast(u16, (__bf16)x); }
__device__ __forceinline__ float bf2f(u16 x) { return __uint_as_float(((u32)x) << 16); }

// ------------------------------------------------------------------ GEMM ---
// C[M][N] = A[M][K] * Bt[N][K]^T, bf16 inputs, fp32 MFMA accumulation, bf16
// output.  128x128 output tile, BK = 64, 4 waves (2x2) of 64x64, each wave a
// 4x4 grid of v_mfma_f32_16x16x32_bf16.  A and B tiles are staged by
// global_load_lds_dwordx4 (LDS-DMA, 1 KiB per wave-instruction) into a
// double-buffered, XOR-swizzled [128][64] image (swizzle applied on the
// global SOURCE address, LDS written lane-linear); fragments are read with
// conflict-free ds_read_b128.  64 KiB LDS -> 2 workgroups per CU.
constexpr int GBM = 128, GBN = 128, GBK = 64, GNT = 256;
constexpr int kGemmLds = 2 * 2 * GBM * GBK * 2;  // [buf][A|B][128][64] bf16

typedef __attribute__((address_space(3))) char lds_t;

__device__ __forceinline__ void glds16(const void* g, lds_t* l) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

__global__ __launch_bounds__(GNT, 2) void k_gemm_bf16_tn(const u16* __restrict__ A, const u16* __restrict__ Bt,
                                                         u16* __restrict__ C, int M, int N, int K, WorkQueue* q,
                                                         const PartTable* table, u32 mode, u32 me, u64* cnt,
                                                         u32 inst_per_tile, u32 refs_per_tile, u32 miss_per_tile,
                                                         u32* status) {
  __shared__ __attribute__((aligned(16))) char smem[kGemmLds + 16];
  lds_t* lds = (lds_t*)smem;
  int* s_slot = (int*)(smem + kGemmLds);
  const u32 xcc = xcc_id();
  // Ownership is decided by thread 0 inside grab_unit (workgroup-uniform).
  u64 t_last = __builtin_amdgcn_s_memtime();
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int tiles_m = M / GBM, tiles_n = N / GBN, ntiles = tiles_m * tiles_n;
  const int nk = K / GBK;
  constexpr int GROUP_M = 8;

  // Per-lane staging geometry: this wave loads chunks c = wid*4 + j (8 rows of
  // 128 B each); lane -> row 8c + lane/8, LDS slot lane%8, global k-chunk
  // (slot ^ (row & 7)).
  int srow[4], scol[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = wid * 4 + j;
    srow[j] = 8 * c + (lane >> 3);
    scol[j] = (((lane & 7) ^ (srow[j] & 7)) * 8);
  }

  for (;;) {
    const int t = grab_unit(q, table, mode, me, xcc, s_slot, (u32)ntiles);
    if (t < 0) break;
    // L2-friendly grouped order (GROUP_M row panels share B column panels).
    const int in_group = GROUP_M * tiles_n;
    const int g = t / in_group;
    const int first_m = g * GROUP_M;
    const int gsz = min(tiles_m - first_m, GROUP_M);
    const int tm = first_m + (t % in_group) % gsz;
    const int tn = (t % in_group) / gsz;
    const u16* Ab = A + (size_t)tm * GBM * K;
    const u16* Bb = Bt + (size_t)tn * GBN * K;

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto stage = [&](int buf, int kt) {
      lds_t* la = lds + buf * (2 * GBM * GBK * 2);
      lds_t* lb = la + GBM * GBK * 2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = wid * 4 + j;
        glds16(Ab + (size_t)srow[j] * K + kt * GBK + scol[j], la + c * 1024);
        glds16(Bb + (size_t)srow[j] * K + kt * GBK + scol[j], lb + c * 1024);
      }
    };

    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
      const lds_t* la = lds + cur * (2 * GBM * GBK * 2);
      const lds_t* lb = la + GBM * GBK * 2;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 a[4], b[4];
        const int chunk = s * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ra = wr * 64 + i * 16 + (lane & 15);
          a[i] = *(const __attribute__((address_space(3))) bf16x8*)(la + ra * 128 + ((chunk ^ (ra & 7)) << 4));
          const int rb = wc * 64 + i * 16 + (lane & 15);
          b[i] = *(const __attribute__((address_space(3))) bf16x8*)(lb + rb * 128 + ((chunk ^ (rb & 7)) << 4));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      cur ^= 1;
    }
    // Epilogue: D(row=(lane>>4)*4+r, col=lane&15) per 16x16 block.
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = tm * GBM + wr * 64 + i * 16 + (lane >> 4) * 4;
        const int n = tn * GBN + wc * 64 + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) C[(size_t)(m + r) * N + n] = f2bf(acc[i][j][r]);
      }
    count_unit(cnt, me, xcc, inst_per_tile, &t_last, refs_per_tile, miss_per_tile, q);
  }
  finish(q, status);
}

// ------------------------------------------------------------ HBM stream ---
// dst = src (float4 copy), 16 B per lane, 16 loads in flight per thread: one
// 256-thread workgroup per CU keeps 64 KiB of reads in flight (enough for
// HBM3E at ~2 us loaded latency) while occupying only one wave slot per SIMD,
// so a co-resident GEMM keeps its two waves/SIMD (VGPR budget 512/SIMD: GEMM
// 2x136 + stream 80 + reduce 64 + gemv 96 = 512 fits; the old 4 WG/CU grids did not).
constexpr int SNT = 256, SUNROLL = 16, RUNROLL = 6;

__global__ __launch_bounds__(SNT) void k_stream_copy(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                                    u64 n4, u32 chunk4, WorkQueue* q, const PartTable* table, u32 mode,
                                                    u32 me, u64* cnt, u32* status) {
  __shared__ int s_slot[4];
  const u32 xcc = xcc_id();
  // Ownership is decided by thread 0 inside grab_unit (workgroup-uniform).
  u64 t_last = __builtin_amdgcn_s_memtime();
  const u32 nchunks = (u32)((n4 + chunk4 - 1) / chunk4);
  // 16 B/lane: one load + one store wave-instruction per 1 KiB moved; every
  // line is a fill (streaming, no reuse).
  const u64 lines = (u64)chunk4 * 16 / 128;
  const u64 inst = (u64)chunk4 * 2 / 64 + 8;
  for (;;) {
    const int c = grab_unit(q, table, mode, me, xcc, s_slot, nchunks);
    if (c < 0) break;
    const u64 base = (u64)c * chunk4;
    const u64 end = min(base + chunk4, n4);
    for (u64 i = base + threadIdx.x; i < end; i += (u64)SNT * SUNROLL) {
      f32x4 v[SUNROLL];
#pragma unroll
      for (int k = 0; k < SUNROLL; ++k) {
        const u64 idx = i + (u64)k * SNT;
        if (idx < end) v[k] = __builtin_nontemporal_load(src + idx);
      }
#pragma unroll
      for (int k = 0; k < SUNROLL; ++k) {
        const u64 idx = i + (u64)k * SNT;
        if (idx < end) __builtin_nontemporal_store(v[k], dst + idx);
      }
    }
    count_unit(cnt, me, xcc, inst, &t_last, 2 * lines, 2 * lines, q);
  }
  finish(q, status);
}

// ------------------------------------------------- reduce-copy (all-reduce) -
// out = a + b on bf16 (the traffic shape of a ring all-reduce step: two reads
// and one write per element).  Used as the collective tenant on one GPU; on
// N > 1 GPUs the tenant issues RCCL all-reduce over xGMI instead.
__global__ __launch_bounds__(SNT) void k_reduce_bf16(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                    u32x4* __restrict__ out, u64 n8, u32 chunk8, WorkQueue* q,
                                                    const PartTable* table, u32 mode, u32 me, u64* cnt,
                                                    u32* status) {
  __shared__ int s_slot[4];
  const u32 xcc = xcc_id();
  // Ownership is decided by thread 0 inside grab_unit (workgroup-uniform).
  u64 t_last = __builtin_amdgcn_s_memtime();
  const u32 nchunks = (u32)((n8 + chunk8 - 1) / chunk8);
  const u64 lines = (u64)chunk8 * 16 / 128;
  const u64 inst = (u64)chunk8 * 3 / 64 + (u64)chunk8 * 16 / 64;
  for (;;) {
    const int c = grab_unit(q, table, mode, me, xcc, s_slot, nchunks);
    if (c < 0) break;
    const u64 base = (u64)c * chunk8, end = min(base + chunk8, n8);
    for (u64 i = base + threadIdx.x; i < end; i += (u64)SNT * RUNROLL) {
      u32x4 x[RUNROLL], y[RUNROLL];
#pragma unroll
      for (int k = 0; k < RUNROLL; ++k) {
        const u64 idx = i + (u64)k * SNT;
        if (idx < end) {
          x[k] = __builtin_nontemporal_load(a + idx);
          y[k] = __builtin_nontemporal_load(b + idx);
        }
      }
#pragma unroll
      for (int k = 0; k < RUNROLL; ++k) {
        const u64 idx = i + (u64)k * SNT;
        if (idx >= end) continue;
        const u32* px = (const u32*)&x[k];
        const u32* py = (const u32*)&y[k];
        u32x4 r;
        u32* pr = (u32*)&r;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float lo = bf2f((u16)(px[w] & 0xffff)) + bf2f((u16)(py[w] & 0xffff));
          const float hi = bf2f((u16)(px[w] >> 16)) + bf2f((u16)(py[w] >> 16));
          pr[w] = (u32)f2bf(lo) | ((u32)f2bf(hi) << 16);
        }
        __builtin_nontemporal_store(r, out + idx);
      }
    }
    count_unit(cnt, me, xcc, inst, &t_last, 3 * lines, 3 * lines, q);
  }
  finish(q, status);
}

// --------------------------------------------------------------- GEMV -----
// y[R] = W[R][K] x[K] (bf16 in, fp32 out): the latency-critical "idle" tenant
// request (a decode-step sized matvec).  A wave owns 4 rows; each lane streams
// 16 B per row per 512-column chunk straight into VGPRs, GV_U chunks (4 rows
// x GV_U W loads + GV_U x loads) in flight before the first use -- no LDS
// round trip, no per-load guards (rows past R are clamped, not branched).
constexpr int GV_U = 2;

__device__ __forceinline__ float dot8(const u32x4 w, const u32x4 v) {
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    s += __uint_as_float(w[e] << 16) * __uint_as_float(v[e] << 16);
    s += __uint_as_float(w[e] & 0xffff0000u) * __uint_as_float(v[e] & 0xffff0000u);
  }
  return s;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 8))) void k_gemv_bf16(const u16* __restrict__ W, const u16* __restrict__ x,
                                                  float* __restrict__ y, int R, int K, WorkQueue* q,
                                                  const PartTable* table, u32 mode, u32 me, u64* cnt,
                                                  u32* status) {
  __shared__ int s_slot[4];
  const u32 xcc = xcc_id();
  // Ownership is decided by thread 0 inside grab_unit (workgroup-uniform).
  u64 t_last = __builtin_amdgcn_s_memtime();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const u32 nchunks = (u32)((R + 15) / 16);  // 16 rows per unit (4 per wave)
  const u64 lines = (u64)16 * K * 2 / 128;
  const int nk = K / 512;  // 512 columns per wave-wide chunk (8 per lane)
  const u32x4* xv = (const u32x4*)x;
  for (;;) {
    const int c = grab_unit(q, table, mode, me, xcc, s_slot, nchunks);
    if (c < 0) break;
    const int row0 = c * 16 + wid * 4;
    const u32x4* wr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) wr[r] = (const u32x4*)(W + (size_t)min(row0 + r, R - 1) * K);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int kc = 0;
    for (; kc + GV_U <= nk; kc += GV_U) {
      u32x4 xr[GV_U], wv[GV_U][4];
#pragma unroll
      for (int u = 0; u < GV_U; ++u) {
        const int k = (kc + u) * 64 + lane;
        xr[u] = xv[k];
#pragma unroll
        for (int r = 0; r < 4; ++r) wv[u][r] = __builtin_nontemporal_load(wr[r] + k);
      }
#pragma unroll
      for (int u = 0; u < GV_U; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] += dot8(wv[u][r], xr[u]);
    }
    for (; kc < nk; ++kc) {
      const int k = kc * 64 + lane;
      const u32x4 xr = xv[k];
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] += dot8(__builtin_nontemporal_load(wr[r] + k), xr);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float s = acc[r];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
      if (lane == 0 && row0 + r < R) y[row0 + r] = s;
    }
    count_unit(cnt, me, xcc, (u64)16 * (K / 512 + 8), &t_last, lines, lines, q);
  }
  finish(q, status);
}

// ------------------------------------------------------------- census ------
// Records (XCC_ID, HW_ID) per workgroup: verifies the workgroup->XCD dealing
// and that XCD gating confines a kernel to its partitions.
__global__ void k_census(u32* out, const PartTable* table, u32 mode, u32 me) {
  const u32 xcc = xcc_id();
  const bool ok = owns(table, mode, me, xcc);
  if (threadIdx.x == 0) {
    out[blockIdx.x * 4 + 0] = xcc;
    out[blockIdx.x * 4 + 1] = hw_id();
    out[blockIdx.x * 4 + 2] = ok ? 1u : 0u;
    out[blockIdx.x * 4 + 3] = 0xC0FFEEu;
  }
  if (ok) {  // keep the workgroup resident a little so dealing is visible
    u64 t = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t < 2000) __builtin_amdgcn_s_sleep(1);
  }
}

}  // namespace gpbs_hip

// ---------------------------------------------------------------- C ABI ----
using namespace gpbs_hip;

extern "C" {

int gpbs_hip_gemm_bf16(const void* A, const void* Bt, void* C, int M, int N, int K, void* q, const void* table,
                       unsigned mode, unsigned me, void* cnt, void* status, int grid, hipStream_t s) {
  if (M % GBM || N % GBN || K % GBK || M <= 0 || N <= 0 || K <= 0) return -22;
  const int ntiles = (M / GBM) * (N / GBN);
  if (grid <= 0) grid = 256 * 2;
  if (grid > ntiles) grid = ntiles;
  // Model: per tile 8192 MFMA + ds_read/glds/epilogue issue; refs = A+B
  // panels in 128-B lines; fills = compulsory bytes spread over the tiles.
  const u32 inst = (u32)((GBM / 16) * (GBN / 16) * (K / 32) * 2 + (K / GBK) * 32 + 64);
  const u32 refs = (u32)(((u64)(GBM + GBN) * K * 2) / 128);
  const u32 miss = (u32)((((u64)M + N) * K * 2 / 128) / ntiles + (u64)GBM * GBN * 2 / 128);
  hipLaunchKernelGGL(k_gemm_bf16_tn, dim3(grid), dim3(GNT), 0, s, (const u16*)A, (const u16*)Bt, (u16*)C, M, N, K,
                     (WorkQueue*)q, (const PartTable*)table, mode, me, (u64*)cnt, inst, refs, miss, (u32*)status);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_stream_copy(const void* src, void* dst, unsigned long long bytes, unsigned chunk_bytes, void* q,
                         const void* table, unsigned mode, unsigned me, void* cnt, void* status, int grid, hipStream_t s) {
  if (bytes % 16 || chunk_bytes % 16 || chunk_bytes == 0) return -22;
  if (grid <= 0) grid = 256;  // one workgroup per CU (see SUNROLL)
  hipLaunchKernelGGL(k_stream_copy, dim3(grid), dim3(SNT), 0, s, (const f32x4*)src, (f32x4*)dst, bytes / 16,
                     chunk_bytes / 16, (WorkQueue*)q, (const PartTable*)table, mode, me, (u64*)cnt, (u32*)status);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_reduce_bf16(const void* a, const void* b, void* out, unsigned long long bytes, unsigned chunk_bytes,
                         void* q, const void* table, unsigned mode, unsigned me, void* cnt, void* status, int grid, hipStream_t s) {
  if (bytes % 16 || chunk_bytes % 16 || chunk_bytes == 0) return -22;
  if (grid <= 0) grid = 256;
  hipLaunchKernelGGL(k_reduce_bf16, dim3(grid), dim3(SNT), 0, s, (const u32x4*)a, (const u32x4*)b, (u32x4*)out,
                     bytes / 16, chunk_bytes / 16, (WorkQueue*)q, (const PartTable*)table, mode, me, (u64*)cnt, (u32*)status);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_gemv_bf16(const void* W, const void* x, void* y, int R, int K, void* q, const void* table, unsigned mode,
                       unsigned me, void* cnt, void* status, int grid, hipStream_t s) {
  if (K % 512 || R <= 0) return -22;
  if (grid <= 0) grid = (R + 15) / 16;
  if (grid > 256) grid = 256;
  hipLaunchKernelGGL(k_gemv_bf16, dim3(grid), dim3(256), 0, s, (const u16*)W, (const u16*)x, (float*)y, R, K,
                     (WorkQueue*)q, (const PartTable*)table, mode, me, (u64*)cnt, (u32*)status);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_census(void* out, int blocks, const void* table, unsigned mode, unsigned me, hipStream_t s) {
  hipLaunchKernelGGL(k_census, dim3(blocks), dim3(64), 0, s, (u32*)out, (const PartTable*)table, mode, me);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // extern "C"
