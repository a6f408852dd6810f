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
__device__ __forceinline__ int grab_unit_x(WorkQueue* q, const PartTable* table, u32 mode, u32 me, u32 xcc,
                                           int* s_slot, u32 total) {
  if (threadIdx.x == 0) {
    int u = -1;
    hold_wait(table, mode);
    const u32 per = (total + kXcds - 1) / kXcds;
    for (u32 spins = 0;; ++spins) {
      if (owns(table, mode, me, xcc)) {
        for (u32 k = 0; k < (u32)kXcds; ++k) {
          const u32 r = (xcc + k) & (kXcds - 1);
          const u32 lo = r * per, hi = min(lo + per, total);
          if (lo >= hi) continue;
          if (__hip_atomic_load(&q->xnext[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= hi - lo) continue;
          const u32 t = atomicAdd(&q->xnext[r], 1u);
          if (t < hi - lo) {
            u = (int)(lo + t);
            atomicAdd(&q->next, 1u);
            break;
          }
        }
        break;
      }
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
  finish(q, status, (u32)ntiles);
}

// -------------------------------------------------------- GEMM 256x256 ----
// The fast path for M, N % 256 == 0 (the co-run GEMM tenant): 256x256 output
// tile per workgroup, BK = 64, 8 waves as 2(M) x 4(N), 128x64 per wave, one
// workgroup per CU (128 KiB LDS).  Halving the A/B panel traffic per FLOP vs
// the 128x128 kernel matters twice here: solo throughput, and how hard the
// GEMM leans on the L2 a co-running memory tenant also streams through.
//
// Schedule (8 phases per 2 K-tiles; one phase = one 64x32 C-quadrant x K=64
// = 16 MFMA per wave), per K-tile t in LDS buffer t&1:
//   phase  reads (ds_read_b128)     stages (global_load_lds, 2 per thread)
//   k0     A rows mi=0 (8) + B ni=0 (4)   B-half1 of tile t+1
//   k1     B ni=1 (4)                     A-half1 of tile t+1
//   k2     A rows mi=1 (8)                B-half0 of tile t+2
//   k3     --                             A-half0 of tile t+2, then vmcnt(4)
// A half h = rows 128h.. (read only by waves wr == h), B half h = columns
// 128h.. (waves wc >> 1 == h).  WAR: a buffer half is restaged one phase
// after the phase that last read it (A halves: k2 -> k3, B halves: k1 -> k2);
// every wave's ds_reads of a phase are retired (lgkmcnt(0)) before that
// phase's closing barrier.  RAW: tile t+1 is retired by the counted vmcnt at
// (t, k3) -- only tile t+2's two halves stay in flight across the barrier --
// and first read at (t+1, k0).  Raw s_barrier (no __syncthreads: its fence
// would drain the LDS-DMA queue), all LDS in one __shared__ array.
// LDS image: [buf][A|B][half][128 rows][128 B], 16-B chunk c of row r stored
// at slot c ^ ((r >> 1) & 7): a 16-lane ds_read_b128 group (16 consecutive
// rows, one logical chunk) covers all 16 slots of a 256-B bank row.
constexpr int G2_BM = 256, G2_BK = 64, G2_NT = 512;
constexpr u32 kGemmXRange = 1u << 16;  // mode bit: XCD-range tile queues (grab_unit_x)
constexpr u32 kGemmBlock2D = 1u << 17; // mode bit: 2-D per-XCD tile blocks
// mode bit (host opts bit 23, ungated launches with one unit per workgroup
// only): unit = blockIdx.x, no work-queue atomic.  A diagnostic of what the
// persistent queue -- which gating, parking and relaunch need -- costs a
// solo launch (scripts/gemm_shapes.py); never set by the runners.  Measured
// (profiles/r6/s61_gemm_shapes.jsonl): 4096^3 0.1130 -> 0.1052 ms (1216 ->
// 1306 TF/s; torch.mm 1475 on that box).  The queue costs ~8 us per launch:
// each workgroup waits on three device-scope atomics with returns (its
// grab, the grab that finds the queue empty, the exit count), a memory
// round trip each, at the start and end of the kernel where nothing hides
// them.  At 8192^3 (4 units per workgroup) the two tie.
constexpr u32 kGemmStatic = 1u << 18;
// host: bit 0 = XCD-range tile queues, bit 1 = DEEP prefetch variant, bit 2 =
// staggered wave groups.  Default = staggered, plain queue: interleaved A/B
// in one process at 4096^3 (profiles/kbench_r1.jsonl) measured staggered
// 1155 TF/s vs 1035 unstaggered, deep prefetch 1036 (no gain: the lead was
// not the limit; MFMA busy was 41 % with the groups in lock-step), XCD-range
// queue 946 (dispatch already deals consecutive tiles round-robin over the
// XCDs, giving each XCD two B panels shared 16 ways).  Bit 3 = 2-D per-XCD
// tile blocks (12 panel slices per XCD K-step instead of 18): 1129 vs 1117
// TF/s plain, 1060 with the XCD-range queue (round 2, interleaved, same box;
// torch.mm 1416) -- panel traffic is not what holds the kernel back.
// round 3: the 2-phase kernel, own-A-half staging (profiles/r3/kbench_gemm_k.log); round 4: C
// staged through LDS, +1.1-1.3 % in three processes on two boxes (profiles/r4/kbench_gemm_ldsc_s51_s52.jsonl),
// its full-line stores non-temporal, another +1.0-1.3 % in three processes on two boxes
// (profiles/r4/kbench_gemm_ldsc_nt_s54_s55.jsonl); round 5: + 2-D per-XCD
// tile blocks (bit 3).  Solo that is worth 0.2-0.5 %; in the co-runs,
// where the memory tenants stream through the same L2s, the GEMM keeps its
// panels and runs 13 % faster: 4mix 1.169 -> 1.250, 8mix 1.275 -> 1.340,
// static-se and gpbs alike (profiles/r5/s21_gemm_blocks_ab.txt).
static int g_gemm_opts = 256 | 8192 | 65536 | 131072 | 8;
constexpr int kG2Half = 128 * 128;           // bytes per half-tile
constexpr int kG2Buf = 4 * kG2Half;          // A0 A1 B0 B1
constexpr int kG2Lds = 2 * kG2Buf;           // 128 KiB

__device__ __forceinline__ int g2_swz(int r) { return (r >> 1) & 7; }

// DEEP = 2 variant (staggered): the wr = 1 wave group runs one barrier (half
// a phase) behind wr = 0, so on every SIMD one wave's ds_reads overlap the
// other's MFMA cluster.  With the groups offset, a buffer half is restaged
// only two phases after its last read, and a staged tile is read only after
// a barrier both groups passed after their counted wait.  Staging per K-tile
// t: (t-1,k3) both B halves of t+1, (t,k0) A-half0 of t+1, (t,k1) A-half1
// of t+1, (t,k3) both B halves of t+2 then vmcnt(4) (retires tile t+1).
// DEEP = 3 (host bit 4): DEEP = 2 with both A halves of t+1 staged in k0 --
// the earliest the two-phase rule allows: 1171 vs 1163 TF/s (round 2, same
// process), so the load lead is not what limits the staggered schedule.
// DEEP = 1 variant: all four halves of K-tile t+2 are issued in k2 (B halves)
// and k3 (A halves) -- the earliest the WAR rule allows -- and the k3 wait is
// vmcnt(8), so a whole K-tile stays in flight for four phases (DEEP = 0: one
// half per phase, vmcnt(4), lead 2-6 phases).
// STAMP = 1: diagnostic build (host opts bit 6, never the default) -- lane 0
// of every wave records s_memtime after each barrier of K-tiles
// kStampT0 .. kStampT0 + kStampTiles - 1 into spare LDS (so no vector-memory
// op perturbs the counted vmcnt waits) and copies them to g_gemm_dbg after
// the unit: [wg < kStampWgs][wave][tile][slot], slot 0 = tile start, 1..8 =
// after the tile's 8 barriers, 9 = s_memrealtime at the tile start (100 MHz).
constexpr int kStampT0 = 8, kStampTiles = 16, kStampSlots = 10, kStampWgs = 64, kStampPhWgs = 1024;
__device__ u32* g_gemm_dbg;

template <int DEEP, int STAMP = 0>
__global__ __launch_bounds__(G2_NT, 1) void k_gemm256_bf16_tn(const u16* __restrict__ A, const u16* __restrict__ Bt,
                                                             u16* __restrict__ C, int M, int N, int K, WorkQueue* q,
                                                             const PartTable* table, u32 mode, u32 me, u64* cnt,
                                                             u32 inst_per_tile, u32 refs_per_tile, u32 miss_per_tile,
                                                             u32* status) {
  constexpr int kStampLds = STAMP ? 8 * kStampTiles * kStampSlots * 4 : 0;
  __shared__ __attribute__((aligned(16))) char smem[kG2Lds + 16 + kStampLds];
  lds_t* lds = (lds_t*)smem;
  int* s_slot = (int*)(smem + kG2Lds);
  const u32 xcc = xcc_id();
  u64 t_last = __builtin_amdgcn_s_memtime();
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  u32* st_lds = (u32*)(smem + kG2Lds + 16) + wid * kStampTiles * kStampSlots;
  auto stamp = [&](int t, int slot) {
    if constexpr (STAMP) {
      if (lane == 0 && t >= kStampT0 && t < kStampT0 + kStampTiles)
        st_lds[(t - kStampT0) * kStampSlots + slot] =
            slot == 9 ? (u32)__builtin_amdgcn_s_memrealtime() : (u32)__builtin_amdgcn_s_memtime();
    }
  };
  const int tiles_m = M / G2_BM, tiles_n = N / G2_BM, ntiles = tiles_m * tiles_n;
  const int nt = K / G2_BK;

  // Staging geometry: wave w's glds j writes 1 KiB chunk c = 2w + j of a
  // half-tile = rows 8c .. 8c+7; lane -> row 8c + lane/8, slot lane%8, source
  // chunk slot ^ swz(row).  Same offsets for every half (A or B, h = 0/1).
  int soff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 8 * (2 * wid + j) + (lane >> 3);
    soff[j] = row * K + (((lane & 7) ^ g2_swz(row)) * 8);
  }
  const int l16 = lane & 15, lq = lane >> 4;

  for (;;) {
    const int tile = (mode & kGemmXRange) ? grab_unit_x(q, table, mode, me, xcc, s_slot, (u32)ntiles)
                                          : grab_unit(q, table, mode, me, xcc, s_slot, (u32)ntiles);
    if (tile < 0) break;
    int tm = tile / tiles_n, tn = tile % tiles_n;  // row-major: an XCD range shares A panels
    if ((mode & kGemmBlock2D) && (tiles_m & 3) == 0 && (tiles_n & 1) == 0) {
      // 2-D XCD blocks: the tiles one XCD computes form a (tiles_m/4) x
      // (tiles_n/2) block (4096^3: 4 A + 8 B panels per XCD instead of 2 A +
      // 16 B row-major, or 16 A + 2 B dealt round-robin), so the 32
      // concurrent tiles of an XCD pull 12 panel slices per K-step into its
      // L2 instead of 18.  The XCD of a tile: its range (XCD-range queue), or
      // ticket mod 8 (plain queue: tickets follow the round-robin dispatch).
      const int per = ntiles / kXcds, bm = tiles_m / 4, bn = tiles_n / 2;
      const int g = (mode & kGemmXRange) ? tile / per : tile % kXcds;
      const int j = (mode & kGemmXRange) ? tile % per : tile / kXcds;
      tm = (g >> 1) * bm + j / bn;
      tn = (g & 1) * bn + j % bn;
    }
    const u16* Ab = A + (size_t)tm * G2_BM * K;
    const u16* Bb = Bt + (size_t)tn * G2_BM * K;

    // stage(kind, h, t): kind 0 = A, 1 = B; half h of K-tile t.
    auto stage = [&](int kind, int h, int t) {
      if (t >= nt) return;
      const u16* src = (kind ? Bb : Ab) + (size_t)h * 128 * K + t * G2_BK;
      lds_t* dst = lds + (t & 1) * kG2Buf + (kind * 2 + h) * kG2Half + wid * 2048;
      glds16(src + soff[0], dst);
      glds16(src + soff[1], dst + 1024);
    };
    // Fragment read: 16 rows starting at `r0` of half-tile (kind, h) of
    // buffer b, k-substep s (32 k): lane reads row r0 + l16, logical chunk 4s + lq.
    auto frag = [&](int b, int kind, int h, int r0, int s) -> bf16x8 {
      const int r = r0 + l16;
      const lds_t* p = lds + b * kG2Buf + (kind * 2 + h) * kG2Half + r * 128 + (((4 * s + lq) ^ g2_swz(r)) << 4);
      return *(const __attribute__((address_space(3))) bf16x8*)p;
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Prologue: all of tile 0, the first two halves of tile 1.
    stage(1, 0, 0); stage(0, 0, 0); stage(1, 1, 0); stage(0, 1, 0);
    if (DEEP >= 2) {
      stage(1, 0, 1); stage(1, 1, 1);
      if (nt > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (DEEP) {
      stage(1, 0, 1); stage(1, 1, 1); stage(0, 0, 1); stage(0, 1, 1);
      if (nt > 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      stage(1, 0, 1); stage(0, 0, 1);
      if (nt > 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();

    if (DEEP >= 2 && wr == 1) __builtin_amdgcn_s_barrier();  // start half a phase behind
    const int bh = wc >> 1;          // B half this wave reads
    const int bc = (wc & 1) * 64;    // its 64 columns within the half
    bf16x8 a[4][2], b0[2][2], b1[2][2];
    for (int t = 0; t < nt; ++t) {
      const int buf = t & 1;
      stamp(t, 9);
      stamp(t, 0);
      // ---- k0: quadrant (mi 0, ni 0)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) b0[j][s] = frag(buf, 1, bh, bc + j * 16, s);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s) a[i][s] = frag(buf, 0, wr, i * 16, s);
      if (DEEP == 0) stage(1, 1, t + 1);
      if (DEEP >= 2) stage(0, 0, t + 1);
      if (DEEP == 3) stage(0, 1, t + 1);  // both A halves of t+1 as early as the 2-phase WAR rule allows
      __builtin_amdgcn_s_barrier();
      stamp(t, 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j][s], a[i][s], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
      stamp(t, 2);
      // ---- k1: quadrant (mi 0, ni 1)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) b1[j][s] = frag(buf, 1, bh, bc + 32 + j * 16, s);
      if (DEEP == 0 || DEEP == 2) stage(0, 1, t + 1);
      __builtin_amdgcn_s_barrier();
      stamp(t, 3);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j][s], a[i][s], acc[i][2 + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
      stamp(t, 4);
      // ---- k2: quadrant (mi 1, ni 1)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s = 0; s < 2; ++s) a[i][s] = frag(buf, 0, wr, 64 + i * 16, s);
      if (DEEP < 2) stage(1, 0, t + 2);
      if (DEEP == 1) stage(1, 1, t + 2);
      __builtin_amdgcn_s_barrier();
      stamp(t, 5);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            acc[4 + i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j][s], a[i][s], acc[4 + i][2 + j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
      stamp(t, 6);
      // ---- k3: quadrant (mi 1, ni 0); retire tile t+1
      if (DEEP >= 2) {
        stage(1, 0, t + 2);
        stage(1, 1, t + 2);
        if (t + 2 < nt) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (DEEP) {
        stage(0, 0, t + 2);
        stage(0, 1, t + 2);
        if (t + 2 < nt) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        stage(0, 0, t + 2);
        if (t + 2 < nt) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      stamp(t, 7);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j][s], a[i][s], acc[4 + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
      stamp(t, 8);
    }
    if (DEEP >= 2 && wr == 0) __builtin_amdgcn_s_barrier();  // re-align the groups
    // Epilogue: mfma(B, A) holds C^T per 16x16 block -- lane owns
    // C[m = .. + l16][n = .. + 4 lq + r], r = 0..3: one 8-byte store.
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = tm * G2_BM + wr * 128 + i * 16 + l16;
        const int n = tn * G2_BM + wc * 64 + j * 16 + 4 * lq;
        const u32 lo = (u32)f2bf(acc[i][j][0]) | ((u32)f2bf(acc[i][j][1]) << 16);
        const u32 hi = (u32)f2bf(acc[i][j][2]) | ((u32)f2bf(acc[i][j][3]) << 16);
        *(uint2*)(C + (size_t)m * N + n) = make_uint2(lo, hi);
      }
    if constexpr (STAMP) {
      if (lane == 0 && blockIdx.x < kStampWgs && nt >= kStampT0 + kStampTiles && g_gemm_dbg) {
        u32* dst = g_gemm_dbg + ((size_t)blockIdx.x * 8 + wid) * kStampTiles * kStampSlots;
        for (int i = 0; i < kStampTiles * kStampSlots; ++i) dst[i] = st_lds[i];
      }
    }
    count_unit(cnt, me, xcc, inst_per_tile, &t_last, refs_per_tile, miss_per_tile, q);
  }
  finish(q, status, (u32)ntiles);
}

// ------------------------------- GEMM 256x256, 8 waves, 2 phases per K-tile ---
// Per-barrier stamps of the 4-phase kernel (scripts/gemm_stamps.py,
// profiles/pmc/gemm_stamps_r3.json: 2.385 GHz in-kernel clock, 3996 cycles
// per K-tile) put every one of its 8 barrier intervals at 400-700 cycles
// against 256 cycles of MFMA work (16 MFMAs of one wave per SIMD): a fixed
// ~200-cycle cost per interval (barrier round trip, the MFMA wave's restart)
// that 8 intervals per K-tile pay 8 times.  This variant keeps the tile,
// the LDS image, the staggered wave groups and glds staging, but runs TWO
// phases per K-tile with 32 MFMAs each: phase A = rows 0-63 of the wave's
// 128 x all 64 columns, phase B = rows 64-127 (the 8 B fragments stay in
// registers across both), so a K-tile has 4 barrier intervals.
// Global interval schedule (tile-relative; g0 = wr 0 reads in 0 and 2, g1
// one barrier behind reads in 1 and 3):
//   g0 int 0: read B (8) + A rows 0-63 (8); stage B0, B1, A0 of t+1;
//             vmcnt(6) retires its A1(t) (issued int 2 of t-1)
//   g1 int 1: same reads; stage all four halves of t+1
//   g0 int 2: read A rows 64-127 (8); stage A1 of t+1; vmcnt(2)
//   g1 int 3: same reads; vmcnt(0)
// WAR: a half of buffer (t+1)&1 is restaged only after the barrier that
// follows the lgkmcnt(0) retiring its last read in tile t-1 (B: read in
// ints 0/1, free from 3 of t-1; A0: int 2, free from int 0 of t; A1: int 3,
// free from int 1 of t).  RAW: every issuer's counted vmcnt precedes a
// barrier the reader passes before its read (g0 reads B, A0 of t+1 at int 4:
// g0 retired them at int 2, g1 at int 3; g1 reads A1 at int 5: g0 retired
// it at int 4).  Host opts bit 8.
// BAL (opts bit 12): the stamps put interval 1 at ~1100 cycles against ~700
// for the others -- g1 issues all 8 glds of t+1 there -- so the balanced
// schedule spreads them: g0 int 0: B0, B1 of t+1, vmcnt(4); int 2: A0, A1,
// vmcnt(4) (retires B); end of int 3: vmcnt(2) (retires A0 before g0 reads
// it at int 4).  g1 int 1: B0, B1, A0; int 3: A1, vmcnt(2) (retires B, A0
// before barrier 3|4); end of int 4: vmcnt(0) (A1, read by g1 at int 5).
// WAR: g0's A0/A1 restage at int 2 (free from int 0 / int 1 of t).
// BAL 2 (opts bit 13): A half h is read only by group h, so each group
// stages its OWN A half alone (4 glds per wave) in its R_B interval, and both
// groups stage their share of the B halves in R_A: 4 glds in every read
// interval.  g0 int 0: B0, B1 of t+1; int 2: A0 of t+1, vmcnt(4) (retires
// B); end of int 3: vmcnt(0) (A0 before g0 reads it at int 4).  g1 int 1:
// B0, B1; int 3: A1, vmcnt(4) (B retired before barrier 3|4); end of int 4:
// vmcnt(0) (A1 before g1 reads it at int 5).  WAR: A0 free from int 0 of t,
// A1 from int 1, B from int 3 of t-1.
template <int STAMP, int NTC, int BAL>
__global__ __launch_bounds__(G2_NT, 1) void k_gemm256s2_bf16_tn(const u16* __restrict__ A, const u16* __restrict__ Bt,
                                                               u16* __restrict__ C, int M, int N, int K, WorkQueue* q,
                                                               const PartTable* table, u32 mode, u32 me, u64* cnt,
                                                               u32 inst_per_tile, u32 refs_per_tile,
                                                               u32 miss_per_tile, u32* status) {
  constexpr int kStampLds = STAMP ? 8 * kStampTiles * kStampSlots * 4 : 0;
  __shared__ __attribute__((aligned(16))) char smem[kG2Lds + 16 + kStampLds];
  lds_t* lds = (lds_t*)smem;
  int* s_slot = (int*)(smem + kG2Lds);
  const u32 xcc = xcc_id();
  u64 t_last = __builtin_amdgcn_s_memtime();
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(wid);  // wave-uniform: scalar branches on the group
  const int wr = wu >> 2, wc = wu & 3;
  const int tiles_m = M / G2_BM, tiles_n = N / G2_BM, ntiles = tiles_m * tiles_n;
  const int nt = K / G2_BK;
  u32* st_lds = (u32*)(smem + kG2Lds + 16) + wid * kStampTiles * kStampSlots;
  auto stamp = [&](int t, int slot) {
    if constexpr (STAMP) {
      if (lane == 0 && t >= kStampT0 && t < kStampT0 + kStampTiles)
        st_lds[(t - kStampT0) * kStampSlots + slot] =
            slot == 9 ? (u32)__builtin_amdgcn_s_memrealtime() : (u32)__builtin_amdgcn_s_memtime();
    }
  };
  int soff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 8 * (2 * wid + j) + (lane >> 3);
    soff[j] = row * K + (((lane & 7) ^ g2_swz(row)) * 8);
  }
  // BAL 2: a group stages its own A half alone -- wave wc of the group
  // writes rows 32 wc .. 32 wc + 31 (4 glds)
  int soffa[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 8 * (4 * (wid & 3) + j) + (lane >> 3);
    soffa[j] = row * K + (((lane & 7) ^ g2_swz(row)) * 8);
  }
  const int l16 = lane & 15, lq = lane >> 4;
  const int bh = wc >> 1, bc = (wc & 1) * 64;
  // STAMP: per workgroup s_memrealtime (100 MHz) at kernel entry, loop start,
  // loop end and after the epilogue stores of its first unit
  u32 ph[4] = {0, 0, 0, 0};
  if constexpr (STAMP) ph[0] = (u32)__builtin_amdgcn_s_memrealtime();
  int units_seen = 0;

  for (;;) {
    const int tile = (mode & kGemmStatic) ? (units_seen ? -1 : (int)blockIdx.x)
                     : (mode & kGemmXRange) ? grab_unit_x(q, table, mode, me, xcc, s_slot, (u32)ntiles)
                                            : grab_unit(q, table, mode, me, xcc, s_slot, (u32)ntiles);
    if (tile < 0) break;
    int tm = tile / tiles_n, tn = tile % tiles_n;
    if ((mode & kGemmBlock2D) && (tiles_m & 3) == 0 && (tiles_n & 1) == 0 && ntiles % kXcds == 0) {
      // 2-D per-XCD blocks (as k_gemm256_bf16_tn): an XCD's tiles form a
      // (tiles_m/4) x (tiles_n/2) block, 12 operand-panel slices per K-step
      // in its L2 instead of 18 (PMC: L2 hit rate 0.68 with row-major
      // dealing).  The XCD of a tile: its range (XCD-range queue: the
      // workgroup's own XCD), or ticket mod 8 (plain queue: tickets follow
      // the round-robin dispatch only approximately)
      const int per = ntiles / kXcds;
      const int bm = tiles_m / 4, bn = tiles_n / 2;
      const int g = (mode & kGemmXRange) ? tile / per : tile % kXcds;
      const int jj = (mode & kGemmXRange) ? tile % per : tile / kXcds;
      tm = (g >> 1) * bm + jj / bn;
      tn = (g & 1) * bn + jj % bn;
    }
    const u16* Ab = A + (size_t)tm * G2_BM * K;
    const u16* Bb = Bt + (size_t)tn * G2_BM * K;
    auto stage = [&](int kind, int h, int t) {
      const u16* src = (kind ? Bb : Ab) + (size_t)h * 128 * K + t * G2_BK;
      lds_t* dst = lds + (t & 1) * kG2Buf + (kind * 2 + h) * kG2Half + wid * 2048;
      glds16(src + soff[0], dst);
      glds16(src + soff[1], dst + 1024);
    };
    auto stage_own_a = [&](int t) {  // all of A half wr of K-tile t, by this group
      const u16* src = Ab + (size_t)wr * 128 * K + t * G2_BK;
      lds_t* dst = lds + (t & 1) * kG2Buf + wr * kG2Half + (wid & 3) * 4096;
#pragma unroll
      for (int j = 0; j < 4; ++j) glds16(src + soffa[j], dst + j * 1024);
    };
    auto frag = [&](int b, int kind, int h, int r0, int s) -> bf16x8 {
      const int r = r0 + l16;
      const lds_t* p = lds + b * kG2Buf + (kind * 2 + h) * kG2Half + r * 128 + (((4 * s + lq) ^ g2_swz(r)) << 4);
      return *(const __attribute__((address_space(3))) bf16x8*)p;
    };
    f32x4 acc[8][4];
    f32x16 acc32[4][2];  // BAL 6
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc32[i][j][e] = 0.f;
    // 32x32x16 operand: lane l holds row r0 + l%32, k = 16 s + 8 (l/32) .. +7
    auto frag32 = [&](int b, int kind, int h, int r0, int s) -> bf16x8 {
      const int r = r0 + (lane & 31);
      const lds_t* p = lds + b * kG2Buf + (kind * 2 + h) * kG2Half + r * 128 + (((2 * s + (lane >> 5)) ^ g2_swz(r)) << 4);
      return *(const __attribute__((address_space(3))) bf16x8*)p;
    };
    // prologue: all of tile 0 from every wave, landed and visible
    stage(1, 0, 0); stage(1, 1, 0); stage(0, 0, 0); stage(0, 1, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();  // g1 runs one barrier behind
    if constexpr (STAMP) {
      if (units_seen == 0) ph[1] = (u32)__builtin_amdgcn_s_memrealtime();
    }
    if constexpr (BAL == 6) {
      // BAL 2's schedule and staging on v_mfma_f32_32x32x16_bf16: a phase is
      // 2 (rows) x 2 (cols) blocks of 32x32 x 4 K-steps = 16 MFMAs of 16
      // passes instead of 32 of 8.  Same 16 fragments per phase (LDS traffic
      // per flop is set by the 128x64 wave tile, not the MFMA shape); half
      // the MFMA issues and one accumulator block per 32x32.
      bf16x8 a[2][4], b[2][4];
      for (int t = 0; t < nt; ++t) {
        const int buf = t & 1;
        const bool more = t + 1 < nt;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < 4; ++s) b[j][s] = frag32(buf, 1, bh, bc + j * 32, s);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int s = 0; s < 4; ++s) a[i][s] = frag32(buf, 0, wr, i * 32, s);
        if (more) {
          stage(1, 0, t + 1); stage(1, 1, t + 1);
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][s], a[i][s], acc32[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int s = 0; s < 4; ++s) a[i][s] = frag32(buf, 0, wr, 64 + i * 32, s);
        if (more) {
          stage_own_a(t + 1);
          asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // retires this group's B0/B1(t+1)
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc32[2 + i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][s], a[i][s], acc32[2 + i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // own A half of t+1 before the next R_A
        __builtin_amdgcn_s_barrier();
      }
    } else if constexpr (BAL == 3) {
      // ONE phase per K-tile (2 barriers): a wave reads all 24 fragments of
      // K-tile t, then runs its 64 MFMAs.  Global intervals: g0 reads at 2t,
      // MFMAs at 2t+1; g1 reads at 2t+1, MFMAs at 2t+2.  Buffer (t+1)&1 is
      // free from interval 2t+1 (g1's reads of tile t-1 retired at 2t).
      // Staging of t+1: g0 stages both B halves and its A0 (12 glds) at the
      // top of its MFMA interval and retires them at its end (g0 reads them
      // at 2t+2, g1 the B halves at 2t+3); g1 stages its A1 (4 glds) in its
      // read interval and retires it at the end of its MFMA interval.
      bf16x8 a8[8][2], b4[4][2];
      for (int t = 0; t < nt; ++t) {
        const int buf = t & 1;
        const bool more = t + 1 < nt;
        stamp(t, 9);
        stamp(t, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) b4[j][s2] = frag(buf, 1, bh, bc + j * 16, s2);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) a8[i][s2] = frag(buf, 0, wr, i * 16, s2);
        if (wr == 1 && more) stage_own_a(t + 1);
        __builtin_amdgcn_s_barrier();
        stamp(t, 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (wr == 0 && more) {
          // g0: B halves (both waves' rows: 4 glds per half per wave) and A0
          for (int h = 0; h < 2; ++h) {
            const u16* src = Bb + (size_t)h * 128 * K + (t + 1) * G2_BK;
            lds_t* dst = lds + ((t + 1) & 1) * kG2Buf + (2 + h) * kG2Half + (wid & 3) * 4096;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) glds16(src + soffa[jj], dst + jj * 1024);
          }
          stage_own_a(t + 1);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b4[j][s2], a8[i][s2], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        if (more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        stamp(t, 2);
      }
    } else {
    constexpr int SB = (BAL == 7 || BAL == 8) ? 2 : BAL;  // BAL 7/8: BAL 2's loop, LDS-staged C
    bf16x8 a[4][2], b[4][2];
    for (int t = 0; t < nt; ++t) {
      const int buf = t & 1;
      const bool more = t + 1 < nt;
      stamp(t, 9);
      stamp(t, 0);
      // ---- R_A: B fragments (kept for both phases), A rows 0-63
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) b[j][s2] = frag(buf, 1, bh, bc + j * 16, s2);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) a[i][s2] = frag(buf, 0, wr, i * 16, s2);
      if constexpr (SB == 2) {  // 4 glds per read interval: B halves here, own A half in R_B
        if (more) {
          stage(1, 0, t + 1); stage(1, 1, t + 1);
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      } else if constexpr (SB) {
        // balanced staging: g0 4 + 4 glds, g1 6 + 2 (see the schedule note)
        if (wr == 0) {
          if (more) {
            stage(1, 0, t + 1); stage(1, 1, t + 1);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // retires A0/A1(t) of int 2 of t-1
          } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
        } else if (more) {
          stage(1, 0, t + 1); stage(1, 1, t + 1); stage(0, 0, t + 1);
        }
      } else if (wr == 0) {
        if (more) {
          stage(1, 0, t + 1); stage(1, 1, t + 1); stage(0, 0, t + 1);
          asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      } else if (more) {
        stage(1, 0, t + 1); stage(1, 1, t + 1); stage(0, 0, t + 1); stage(0, 1, t + 1);
      }
      __builtin_amdgcn_s_barrier();
      stamp(t, 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][s2], a[i][s2], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
      stamp(t, 2);
      // ---- R_B: A rows 64-127
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) a[i][s2] = frag(buf, 0, wr, 64 + i * 16, s2);
      if constexpr (SB == 2) {
        if (more) {
          stage_own_a(t + 1);
          asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // retires this group's B0/B1(t+1)
        }
      } else if constexpr (SB) {
        if (wr == 0) {
          if (more) {
            stage(0, 0, t + 1); stage(0, 1, t + 1);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // retires B0/B1(t+1)
          }
        } else if (more) {
          stage(0, 1, t + 1);
          asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // retires B0/B1/A0(t+1)
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      } else if (wr == 0) {
        if (more) {
          stage(0, 1, t + 1);
          asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        }
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      stamp(t, 3);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][s2], a[i][s2], acc[4 + i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if constexpr (SB == 2) {  // end of M_B: the group's own A half of t+1 lands before its next R_A
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if constexpr (SB) {  // end of M_B: g0 retires its A0(t+1), g1 its A1(t+1), before the barrier
        if (wr == 0) {
          if (more) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      __builtin_amdgcn_s_barrier();
      stamp(t, 4);
    }
    }  // BAL != 3
    if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the groups
    if constexpr (STAMP) {
      if (units_seen == 0) ph[2] = (u32)__builtin_amdgcn_s_memrealtime();
    }
    if constexpr (BAL == 6) {
      // mfma32(B, A) holds C^T per 32x32 block: lane owns C[m = .. + l%32][n =
      // .. + 8 g + 4 (l/32) + r], element 4 g + r: one 8-byte store per g
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int m = tm * G2_BM + wr * 128 + i * 32 + (lane & 31);
            const int n = tn * G2_BM + wc * 64 + j * 32 + 8 * g + 4 * (lane >> 5);
            const u32 lo = (u32)f2bf(acc32[i][j][4 * g]) | ((u32)f2bf(acc32[i][j][4 * g + 1]) << 16);
            const u32 hi = (u32)f2bf(acc32[i][j][4 * g + 2]) | ((u32)f2bf(acc32[i][j][4 * g + 3]) << 16);
            *(uint2*)(C + (size_t)m * N + n) = make_uint2(lo, hi);
          }
    } else if constexpr (BAL == 7 || BAL == 8) {
      // C through LDS (the K loop's two buffers are exactly the 256x256 bf16
      // tile): each wave writes its 8-byte fragments at row m, 8-byte chunk
      // n/4 XOR (m & 15), then the workgroup stores 16 rows per pass, each row
      // as 32 contiguous 16-byte stores: full 128-byte lines instead of
      // 32-byte runs.  Banking (MI355X_MICROARCH.md §LDS): a ds_write_b64 is
      // four groups of 16 contiguous lanes on (a/4) mod 32 -- one group is 16
      // rows of one chunk column, and XOR (m & 15) puts them on 16 distinct
      // 8-byte positions of the 128-byte bank row (round 4's XOR 2 (m & 15)
      // used 8: a 2-way conflict on every C write, 2.6 M extra cycles per
      // 4096^3 GEMM); a ds_read_b128 group reads one row's 16 distinct 16-byte
      // slots.  An odd row's two 8-byte chunks of a slot come swapped.
      // Every wave's K-loop reads retired before the re-align barrier above.
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = wr * 128 + i * 16 + l16;
          const int c8 = wc * 16 + j * 4 + lq;
          const u32 lo = (u32)f2bf(acc[i][j][0]) | ((u32)f2bf(acc[i][j][1]) << 16);
          const u32 hi = (u32)f2bf(acc[i][j][2]) | ((u32)f2bf(acc[i][j][3]) << 16);
          *(__attribute__((address_space(3))) u32x2*)(lds + m * 512 + ((c8 ^ (m & 15)) << 3)) = u32x2{lo, hi};
        }
      __syncthreads();
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        const int row = p * 16 + (tid >> 5), c16 = tid & 31;
        u32x4 v = *(const __attribute__((address_space(3))) u32x4*)(lds + row * 512 + (((2 * c16) ^ (row & 14)) << 3));
        if (row & 1) v = u32x4{v.z, v.w, v.x, v.y};
        u32x4* dst = (u32x4*)(C + (size_t)(tm * G2_BM + row) * N + tn * G2_BM + c16 * 8);
        if constexpr (BAL == 8) {  // streaming full-line stores (opts bit 17)
          __builtin_nontemporal_store(v, dst);
        } else {
          *dst = v;
        }
      }
      __syncthreads();  // the next tile's prologue restages buffer 0
    } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = tm * G2_BM + wr * 128 + i * 16 + l16;
        const int n = tn * G2_BM + wc * 64 + j * 16 + 4 * lq;
        const u32 lo = (u32)f2bf(acc[i][j][0]) | ((u32)f2bf(acc[i][j][1]) << 16);
        const u32 hi = (u32)f2bf(acc[i][j][2]) | ((u32)f2bf(acc[i][j][3]) << 16);
        if constexpr (NTC) {  // streaming store: C does not sit dirty in L2 for the end-of-kernel writeback
          __builtin_nontemporal_store((u64)lo | ((u64)hi << 32), (u64*)(C + (size_t)m * N + n));
        } else {
          *(uint2*)(C + (size_t)m * N + n) = make_uint2(lo, hi);
        }
      }
    }  // BAL != 6
    if constexpr (STAMP) {
      if (units_seen == 0) {
        ph[3] = (u32)__builtin_amdgcn_s_memrealtime();
        if (tid == 0 && g_gemm_dbg && blockIdx.x < kStampPhWgs) {
          u32* dp = g_gemm_dbg + kStampWgs * 8 * kStampTiles * kStampSlots + blockIdx.x * 4;
          for (int k = 0; k < 4; ++k) dp[k] = ph[k];
        }
      }
      if (lane == 0 && blockIdx.x < kStampWgs && nt >= kStampT0 + kStampTiles && g_gemm_dbg) {
        u32* dst = g_gemm_dbg + ((size_t)blockIdx.x * 8 + wid) * kStampTiles * kStampSlots;
        for (int i = 0; i < kStampTiles * kStampSlots; ++i) dst[i] = st_lds[i];
      }
    }
    ++units_seen;
    if (!(mode & kGemmStatic)) count_unit(cnt, me, xcc, inst_per_tile, &t_last, refs_per_tile, miss_per_tile, q);
  }
  if (!(mode & kGemmStatic)) finish(q, status, (u32)ntiles);  // (static: the queue was never touched)
}

// ------------------------- GEMM 256x256, 8 waves, pipelined fragments ----
// The 2-phase kernel's four barrier intervals per K-tile cost ~200 cycles
// each on top of 512 MFMA cycles (stamps, see above): MFMA busy 0.53.  This
// variant keeps the 8 waves (2 per SIMD: each SIMD's two waves cover each
// other's LDS latency), the 128x64 wave tile, the LDS image, its swizzle and
// the LDS-staged C epilogue of BAL 8, but runs ONE barrier per K-tile and
// reads fragments into a second register set while the current set's MFMAs
// run (sched_group_barrier interleaves one ds_read per two MFMAs):
//   substep (t, 0): 32 MFMA on X  | reads of (t, 1) -> Y
//   substep (t, 1): 16 MFMA on Y;  lgkmcnt(0) (no read of buffer t&1 left),
//                   vmcnt(0) (this wave's part of tile t+1 landed);
//                   s_barrier (tile t+1 in LDS; buffer t&1 free everywhere);
//                   stage tile t+2 -> buffer t&1 (8 glds);
//                   16 MFMA on Y  | reads of (t+1, 0) -> X
// Registers: 128 accumulators + 64 fragment registers (one A set, re-read
// block by block behind its MFMAs; two B sets).  The tile t+2
// load has one K-tile (~2000 MFMA cycles per SIMD) to land.  Host opts bit
// 18.
__global__ __launch_bounds__(G2_NT, 1) void k_gemm256p_bf16_tn(const u16* __restrict__ A, const u16* __restrict__ Bt,
                                                              u16* __restrict__ C, int M, int N, int K, WorkQueue* q,
                                                              const PartTable* table, u32 mode, u32 me, u64* cnt,
                                                              u32 inst_per_tile, u32 refs_per_tile, u32 miss_per_tile,
                                                              u32* status) {
  __shared__ __attribute__((aligned(16))) char smem[kG2Lds + 16];
  lds_t* lds = (lds_t*)smem;
  int* s_slot = (int*)(smem + kG2Lds);
  const u32 xcc = xcc_id();
  u64 t_last = __builtin_amdgcn_s_memtime();
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  const int wr = wu >> 2, wc = wu & 3;
  const int tiles_n = N / G2_BM, ntiles = (M / G2_BM) * tiles_n;
  const int nt = K / G2_BK;
  int soff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 8 * (2 * wid + j) + (lane >> 3);
    soff[j] = row * K + (((lane & 7) ^ g2_swz(row)) * 8);
  }
  const int l16 = lane & 15, lq = lane >> 4;
  const int bh = wc >> 1, bc = (wc & 1) * 64;
  for (;;) {
    const int tile = grab_unit(q, table, mode, me, xcc, s_slot, (u32)ntiles);
    if (tile < 0) break;
    const int tm = tile / tiles_n, tn = tile % tiles_n;
    const u16* Ab = A + (size_t)tm * G2_BM * K;
    const u16* Bb = Bt + (size_t)tn * G2_BM * K;
    auto stage_tile = [&](int t) {  // this wave's 2 KiB of each of the 4 half-tiles of K-tile t
#pragma unroll
      for (int kind = 0; kind < 2; ++kind)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const u16* src = (kind ? Bb : Ab) + (size_t)h * 128 * K + t * G2_BK;
          lds_t* dst = lds + (t & 1) * kG2Buf + (kind * 2 + h) * kG2Half + wid * 2048;
          glds16(src + soff[0], dst);
          glds16(src + soff[1], dst + 1024);
        }
    };
    auto frag = [&](int b, int kind, int h, int r0, int s) -> bf16x8 {
      const int r = r0 + l16;
      const lds_t* p = lds + b * kG2Buf + (kind * 2 + h) * kG2Half + r * 128 + (((4 * s + lq) ^ g2_swz(r)) << 4);
      return *(const __attribute__((address_space(3))) bf16x8*)p;
    };
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // One A set (an A fragment is re-read into its registers right after its
    // 4 MFMAs issued) and two B sets (B fragments feed all 8 row blocks).
    bf16x8 a[8], b0[4], b1[4];
    // prologue: tiles 0 and 1 in flight; tile 0 landed and visible; (0, 0) read
    stage_tile(0);
    if (nt > 1) {
      stage_tile(1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 4; ++j) b0[j] = frag(0, 1, bh, bc + j * 16, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = frag(0, 0, wr, i * 16, 0);
    for (int t = 0; t < nt; ++t) {
      const int buf = t & 1;
      const bool more = t + 1 < nt;
      // ---- substep 0: 32 MFMA on (b0, a); reads of (t, 1): b1, then a[i]
      //      behind row block i's MFMAs
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j) b1[j] = frag(buf, 1, bh, bc + j * 16, 1);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j], a[i], acc[i][j], 0, 0, 0);
        a[i] = frag(buf, 0, wr, i * 16, 1);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read (b1)
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);  // 3 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read (a[i])
      }
      __builtin_amdgcn_sched_barrier(0);
      // ---- substep 1, first half: 16 MFMA on (b1, a[0..3])
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every read of buffer t&1 by this wave retired
      if (more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of tile t+1 landed
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < nt) stage_tile(t + 2);
      __builtin_amdgcn_sched_barrier(0);
      // ---- substep 1, second half: 16 MFMA on (b1, a[4..7]); reads of
      //      (t+1, 0): b0 and a[0..3] now, a[i] behind row block i's MFMAs
      // (after the last K-tile these read the other buffer's stale tile,
      // unused: straight-line code lets the compiler count lgkmcnt)
#pragma unroll
      for (int j = 0; j < 4; ++j) b0[j] = frag(buf ^ 1, 1, bh, bc + j * 16, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag(buf ^ 1, 0, wr, i * 16, 0);
#pragma unroll
      for (int i = 4; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a[i], acc[i][j], 0, 0, 0);
        a[i] = frag(buf ^ 1, 0, wr, i * 16, 0);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read (b0, a[0..3])
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read (a[4..7])
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's K-loop reads retired: the buffers take C
    __builtin_amdgcn_sched_barrier(0);
    // Epilogue: BAL 8's (C staged through the LDS at XOR (m & 15), full-line
    // non-temporal stores)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = wr * 128 + i * 16 + l16;
        const int c8 = wc * 16 + j * 4 + lq;
        const u32 lo = (u32)f2bf(acc[i][j][0]) | ((u32)f2bf(acc[i][j][1]) << 16);
        const u32 hi = (u32)f2bf(acc[i][j][2]) | ((u32)f2bf(acc[i][j][3]) << 16);
        *(__attribute__((address_space(3))) u32x2*)(lds + m * 512 + ((c8 ^ (m & 15)) << 3)) = u32x2{lo, hi};
      }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const int row = p * 16 + (tid >> 5), c16 = tid & 31;
      u32x4 v = *(const __attribute__((address_space(3))) u32x4*)(lds + row * 512 + (((2 * c16) ^ (row & 14)) << 3));
      if (row & 1) v = u32x4{v.z, v.w, v.x, v.y};
      u32x4* dst = (u32x4*)(C + (size_t)(tm * G2_BM + row) * N + tn * G2_BM + c16 * 8);
      __builtin_nontemporal_store(v, dst);
    }
    __syncthreads();  // the next tile's prologue restages buffer 0
    count_unit(cnt, me, xcc, inst_per_tile, &t_last, refs_per_tile, miss_per_tile, q);
  }
  finish(q, status, (u32)ntiles);
}

// The same schedule with the fragment reads as inline-asm ds_read_b128 and
// counted lgkmcnt waits (the compiler's waits above are lgkmcnt(0) at both
// substep boundaries, stalling the two waves of a SIMD together).  Reads
// are issued in one fixed order per substep -- B set, then A blocks 0..7 --
// so block i of the next substep needs only the reads up to its own: a
// substep's waits are lgkmcnt(7) (B + A block 0 of the previous substep's
// 12), then lgkmcnt(11) for each later block of substep 0 (its 4 B + i A
// reads of substep 1 issued since) and lgkmcnt(7 - i) in substep 1.  An
// empty asm "+v" on each operand after its wait keeps the MFMA behind it.
// Host opts bit 19.
#define GPBS_DSR(dst, p) asm volatile("ds_read_b128 %0, %1" : "=v"(dst) : "v"((u32)(size_t)(p)))
#define GPBS_TOUCH(x) asm volatile("" : "+v"(x))
#define W4J_DSR(dst, base, off) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(off))
#define GPBS_LGKM(n) asm volatile("s_waitcnt lgkmcnt(" #n ")" ::: "memory")
__global__ __launch_bounds__(G2_NT, 1) void k_gemm256p2_bf16_tn(const u16* __restrict__ A, const u16* __restrict__ Bt,
                                                               u16* __restrict__ C, int M, int N, int K, WorkQueue* q,
                                                               const PartTable* table, u32 mode, u32 me, u64* cnt,
                                                               u32 inst_per_tile, u32 refs_per_tile, u32 miss_per_tile,
                                                               u32* status) {
  __shared__ __attribute__((aligned(16))) char smem[kG2Lds + 16];
  lds_t* lds = (lds_t*)smem;
  int* s_slot = (int*)(smem + kG2Lds);
  const u32 xcc = xcc_id();
  u64 t_last = __builtin_amdgcn_s_memtime();
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  const int wr = wu >> 2, wc = wu & 3;
  const int tiles_n = N / G2_BM, ntiles = (M / G2_BM) * tiles_n;
  const int nt = K / G2_BK;
  int soff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 8 * (2 * wid + j) + (lane >> 3);
    soff[j] = row * K + (((lane & 7) ^ g2_swz(row)) * 8);
  }
  const int l16 = lane & 15, lq = lane >> 4;
  const int bh = wc >> 1, bc = (wc & 1) * 64;
  for (;;) {
    const int tile = grab_unit(q, table, mode, me, xcc, s_slot, (u32)ntiles);
    if (tile < 0) break;
    const int tm = tile / tiles_n, tn = tile % tiles_n;
    const u16* Ab = A + (size_t)tm * G2_BM * K;
    const u16* Bb = Bt + (size_t)tn * G2_BM * K;
    auto stage_tile = [&](int t) {
#pragma unroll
      for (int kind = 0; kind < 2; ++kind)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const u16* src = (kind ? Bb : Ab) + (size_t)h * 128 * K + t * G2_BK;
          lds_t* dst = lds + (t & 1) * kG2Buf + (kind * 2 + h) * kG2Half + wid * 2048;
          glds16(src + soff[0], dst);
          glds16(src + soff[1], dst + 1024);
        }
    };
    auto fp = [&](int b, int kind, int h, int r0, int s) -> const lds_t* {
      const int r = r0 + l16;
      return lds + b * kG2Buf + (kind * 2 + h) * kG2Half + r * 128 + (((4 * s + lq) ^ g2_swz(r)) << 4);
    };
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a[8], b0[4], b1[4];
    stage_tile(0);
    if (nt > 1) {
      stage_tile(1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 4; ++j) GPBS_DSR(b0[j], fp(0, 1, bh, bc + j * 16, 0));
#pragma unroll
    for (int i = 0; i < 8; ++i) GPBS_DSR(a[i], fp(0, 0, wr, i * 16, 0));
    for (int t = 0; t < nt; ++t) {
      const int buf = t & 1;
      const bool more = t + 1 < nt;
      // ---- substep 0: (b0, a) of (t, 0); reads of (t, 1): b1, then a[i] behind block i
      __builtin_amdgcn_sched_barrier(0);
      GPBS_LGKM(7);
#pragma unroll
      for (int j = 0; j < 4; ++j) GPBS_TOUCH(b0[j]);
      GPBS_TOUCH(a[0]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j], a[0], acc[0][j], 0, 0, 0);
        GPBS_DSR(b1[j], fp(buf, 1, bh, bc + j * 16, 1));
        __builtin_amdgcn_sched_barrier(0);
      }
      GPBS_DSR(a[0], fp(buf, 0, wr, 0, 1));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 1; i < 8; ++i) {
        GPBS_LGKM(11);
        GPBS_TOUCH(a[i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j], a[i], acc[i][j], 0, 0, 0);
        GPBS_DSR(a[i], fp(buf, 0, wr, i * 16, 1));
        __builtin_amdgcn_sched_barrier(0);
      }
      // ---- substep 1, first half: (b1, a[0..3]) of (t, 1)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i == 0) GPBS_LGKM(7);
        if (i == 1) GPBS_LGKM(6);
        if (i == 2) GPBS_LGKM(5);
        if (i == 3) GPBS_LGKM(4);
        if (i == 0)
#pragma unroll
          for (int j = 0; j < 4; ++j) GPBS_TOUCH(b1[j]);
        GPBS_TOUCH(a[i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      GPBS_LGKM(0);  // every read of buffer t&1 by this wave retired (a[4..7] too)
#pragma unroll
      for (int i = 4; i < 8; ++i) GPBS_TOUCH(a[i]);
      if (more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of tile t+1 landed
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < nt) stage_tile(t + 2);
      __builtin_amdgcn_sched_barrier(0);
      // ---- substep 1, second half: (b1, a[4..7]); reads of (t+1, 0) in the
      //      order b0[0..3], a[0..3] (free), then a[i] behind block i
      //      (after the last K-tile they read the other buffer's stale tile, unused)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[4][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a[4], acc[4][j], 0, 0, 0);
        GPBS_DSR(b0[j], fp(buf ^ 1, 1, bh, bc + j * 16, 0));
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[5][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a[5], acc[5][j], 0, 0, 0);
        GPBS_DSR(a[j], fp(buf ^ 1, 0, wr, j * 16, 0));
        __builtin_amdgcn_sched_barrier(0);
      }
      GPBS_DSR(a[4], fp(buf ^ 1, 0, wr, 64, 0));
      GPBS_DSR(a[5], fp(buf ^ 1, 0, wr, 80, 0));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[6][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a[6], acc[6][j], 0, 0, 0);
      GPBS_DSR(a[6], fp(buf ^ 1, 0, wr, 96, 0));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[7][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a[7], acc[7][j], 0, 0, 0);
      GPBS_DSR(a[7], fp(buf ^ 1, 0, wr, 112, 0));
      __builtin_amdgcn_sched_barrier(0);
    }
    GPBS_LGKM(0);
    __builtin_amdgcn_s_barrier();  // every wave's K-loop reads retired: the buffers take C
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = wr * 128 + i * 16 + l16;
        const int c8 = wc * 16 + j * 4 + lq;
        const u32 lo = (u32)f2bf(acc[i][j][0]) | ((u32)f2bf(acc[i][j][1]) << 16);
        const u32 hi = (u32)f2bf(acc[i][j][2]) | ((u32)f2bf(acc[i][j][3]) << 16);
        *(__attribute__((address_space(3))) u32x2*)(lds + m * 512 + ((c8 ^ (m & 15)) << 3)) = u32x2{lo, hi};
      }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const int row = p * 16 + (tid >> 5), c16 = tid & 31;
      u32x4 v = *(const __attribute__((address_space(3))) u32x4*)(lds + row * 512 + (((2 * c16) ^ (row & 14)) << 3));
      if (row & 1) v = u32x4{v.z, v.w, v.x, v.y};
      u32x4* dst = (u32x4*)(C + (size_t)(tm * G2_BM + row) * N + tn * G2_BM + c16 * 8);
      __builtin_nontemporal_store(v, dst);
    }
    __syncthreads();
    count_unit(cnt, me, xcc, inst_per_tile, &t_last, refs_per_tile, miss_per_tile, q);
  }
  finish(q, status, (u32)ntiles);
}

// ------------------------------------------------ GEMM 256x256, 4 waves ----
// The shape hipBLASLt picks for this GEMM on gfx950 (rocprofv3 kernel trace of
// torch.mm 4096^3, profiles/kbench_r2_w4.md: MT256x256x64, MI16x16, 256
// threads, 130 KiB LDS, one wave per SIMD).  Four waves as 2(M) x 2(N),
// 128x128 per wave = 8x8 blocks of 16x16x32 (256 accumulator registers,
// AGPRs), so a wave reads 32 KiB of fragments per K-tile: 128 KiB per CU
// instead of the 8-wave kernel's 8 x 24 KiB, and ONE barrier per K-tile
// instead of eight.  With one wave per SIMD there is no partner to cover LDS
// latency, so the wave covers it itself: the fragments of the next K-substep
// go into the other register set while this substep's 64 MFMAs run.
// Per K-tile t (LDS buffer t&1; set X = substep (t, 0) already read):
//   read (t, 1) -> Y;  64 MFMA on X;  lgkmcnt(0), vmcnt(0) (tile t+1 landed);
//   s_barrier (every wave done with buffer t&1; tile t+1 in LDS everywhere);
//   stage tile t+2 -> buffer t&1;  read (t+1, 0) -> X;  64 MFMA on Y.
// Same LDS image and swizzle as k_gemm256_bf16_tn (a wave's 4 glds per half
// write rows 32w .. 32w+31).  Host opts bit 5; measured (profiles/
// kbench_r2_w4.md, same process): 1041 TF/s vs 1127 for the staggered 8-wave
// kernel (default) and 1433 for hipBLASLt.  The compiler keeps copying ~96
// accumulator registers AGPR <-> VGPR around every K-tile, and the 16-read /
// 16-glds clumps leave the matrix pipe idle; interleaving them one per MFMA in
// source order (sched_barrier fences) made the copies worse: 896 TF/s.
// Round 6, ROCm 7.2 ISA: the compiler picks the VGPR form of every MFMA here
// (accumulators in VGPRs, 476 registers) and uses the AGPRs as spill space:
// 320 v_accvgpr_read + 544 v_accvgpr_write per unit, 96 + 64 of them inside
// each 64-MFMA block.  Neither `-mllvm -amdgpu-mfma-vgpr-form=0` nor an
// inline asm that clobbers an AGPR moves the accumulators into AGPRs.
// Reaching the library needs the schedule in assembly, not in HIP.
constexpr int G4_NT = 256;

// AS = 1 (host opts bit 20 with bit 5): the MFMAs as inline asm with the
// accumulator tied to AGPRs ("+a"), so the 256 accumulators live in the AGPR
// half of the register file and the fragments in VGPRs -- the split the
// compiler does not choose by itself.  The asm is opaque to the hazard
// recognizer, so the kernel pads the two hazards it creates itself: after
// zeroing the accumulators (v_accvgpr_write -> MFMA SrcC) and after the last
// MFMA (XDL write -> v_accvgpr_read in the epilogue).
template <int AS>
__device__ __forceinline__ void w4_mfma(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  if constexpr (AS) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  } else {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
}

template <int AS>
__global__ __launch_bounds__(G4_NT, 1) void k_gemm256w4_bf16_tn(const u16* __restrict__ A,
                                                               const u16* __restrict__ Bt, u16* __restrict__ C,
                                                               int M, int N, int K, WorkQueue* q,
                                                               const PartTable* table, u32 mode, u32 me, u64* cnt,
                                                               u32 inst_per_tile, u32 refs_per_tile,
                                                               u32 miss_per_tile, u32* status) {
  __shared__ __attribute__((aligned(16))) char smem[kG2Lds + 16];
  lds_t* lds = (lds_t*)smem;
  int* s_slot = (int*)(smem + kG2Lds);
  const u32 xcc = xcc_id();
  u64 t_last = __builtin_amdgcn_s_memtime();
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int tiles_n = N / G2_BM, ntiles = (M / G2_BM) * tiles_n;
  const int nt = K / G2_BK;
  int soff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 8 * (4 * wid + j) + (lane >> 3);
    soff[j] = row * K + (((lane & 7) ^ g2_swz(row)) * 8);
  }
  const int l16 = lane & 15, lq = lane >> 4;
  for (;;) {
    const int tile = grab_unit(q, table, mode, me, xcc, s_slot, (u32)ntiles);
    if (tile < 0) break;
    const int tm = tile / tiles_n, tn = tile % tiles_n;
    const u16* Ab = A + (size_t)tm * G2_BM * K;
    const u16* Bb = Bt + (size_t)tn * G2_BM * K;

    auto stage_tile = [&](int t) {
      if (t >= nt) return;
#pragma unroll
      for (int kind = 0; kind < 2; ++kind)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const u16* src = (kind ? Bb : Ab) + (size_t)h * 128 * K + t * G2_BK;
          lds_t* dst = lds + (t & 1) * kG2Buf + (kind * 2 + h) * kG2Half + wid * 4096;
#pragma unroll
          for (int j = 0; j < 4; ++j) glds16(src + soff[j], dst + j * 1024);
        }
    };
    auto frag = [&](int b, int kind, int h, int r0, int s) -> bf16x8 {
      const int r = r0 + l16;
      const lds_t* p = lds + b * kG2Buf + (kind * 2 + h) * kG2Half + r * 128 + (((4 * s + lq) ^ g2_swz(r)) << 4);
      return *(const __attribute__((address_space(3))) bf16x8*)p;
    };

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (AS) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    bf16x8 xa[8], xb[8], ya[8], yb[8];

    stage_tile(0);
    stage_tile(1);  // nt >= 2 (host: even K-tile count)
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 landed (16 glds per wave per tile)
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int i = 0; i < 8; ++i) xa[i] = frag(0, 0, wr, i * 16, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) xb[j] = frag(0, 1, wc, j * 16, 0);

    for (int t = 0; t < nt; ++t) {
      const int buf = t & 1;
#pragma unroll
      for (int i = 0; i < 8; ++i) ya[i] = frag(buf, 0, wr, i * 16, 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) yb[j] = frag(buf, 1, wc, j * 16, 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) w4_mfma<AS>(acc[i][j], xb[j], xa[i]);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (t + 1 < nt) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      stage_tile(t + 2);
      if (t + 1 < nt) {
#pragma unroll
        for (int i = 0; i < 8; ++i) xa[i] = frag(buf ^ 1, 0, wr, i * 16, 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) xb[j] = frag(buf ^ 1, 1, wc, j * 16, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) w4_mfma<AS>(acc[i][j], yb[j], ya[i]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // (every read of this unit fed an MFMA above; grab_unit's barriers keep
    // the next unit's prologue staging behind all of them)
    if constexpr (AS) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = tm * G2_BM + wr * 128 + i * 16 + l16;
        const int n = tn * G2_BM + wc * 128 + j * 16 + 4 * lq;
        const u32 lo = (u32)f2bf(acc[i][j][0]) | ((u32)f2bf(acc[i][j][1]) << 16);
        const u32 hi = (u32)f2bf(acc[i][j][2]) | ((u32)f2bf(acc[i][j][3]) << 16);
        *(uint2*)(C + (size_t)m * N + n) = make_uint2(lo, hi);
      }
    count_unit(cnt, me, xcc, inst_per_tile, &t_last, refs_per_tile, miss_per_tile, q);
  }
  finish(q, status, (u32)ntiles);
}

// --------------------------- GEMM 256x256, 4 waves, interleaved schedule ---
// k_gemm256w4_bf16_tn<1>'s shape and register split (256 accumulators in
// AGPRs through inline-asm MFMAs, the fragments of two K-substeps in VGPRs),
// with the whole K loop in a fixed issue order: fragment reads are inline-asm
// ds_read_b128 and every MFMA / read / staging load sits between
// sched_barrier fences, so the 16 reads and 16 glds of a substep are spread
// one per MFMA over the first half of its 64 MFMAs instead of issued in
// clumps.  Per K-tile t (buffer b = t & 1, set X = substep (t, 0) in VGPRs):
//   M1: 64 MFMA on X; reads of (t, 1) -> Y behind MFMAs 0, 2, .., 30;
//       lgkmcnt(0), vmcnt(0) (my part of tile t+1 landed), s_barrier
//       (buffer b read by nobody any more; tile t+1 visible everywhere);
//   M2: 64 MFMA on Y; glds of tile t+2 -> buffer b behind MFMAs 1, 3, ..;
//       reads of (t+1, 0) -> X from buffer b^1 behind MFMAs 0, 2, .., 30;
//       lgkmcnt(0) at the next M1 (X landed).
// Epilogue: C staged through LDS, full-line non-temporal stores (as BAL 8);
// 2-D per-XCD tile blocks with opts bit 3.  Host opts bit 21 (with bit 5).
// Measured (profiles/r6/s54, s55, s57; kbench, same process): the AGPR split
// alone lifts the 4-wave kernel from 922 to 1077 TF/s; this issue order to
// 1237-1254, against 1266-1273 for the shipped 8-wave kernel and 1281-1423
// for torch.mm.  Not the default.
__global__ __launch_bounds__(G4_NT, 1) void k_gemm256w4i_bf16_tn(const u16* __restrict__ A,
                                                                const u16* __restrict__ Bt, u16* __restrict__ C,
                                                                int M, int N, int K, WorkQueue* q,
                                                                const PartTable* table, u32 mode, u32 me, u64* cnt,
                                                                u32 inst_per_tile, u32 refs_per_tile,
                                                                u32 miss_per_tile, u32* status) {
  __shared__ __attribute__((aligned(16))) char smem[kG2Lds + 16];
  lds_t* lds = (lds_t*)smem;
  int* s_slot = (int*)(smem + kG2Lds);
  const u32 xcc = xcc_id();
  u64 t_last = __builtin_amdgcn_s_memtime();
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  const int wr = wu >> 1, wc = wu & 1;
  const int tiles_m = M / G2_BM, tiles_n = N / G2_BM, ntiles = tiles_m * tiles_n;
  const int nt = K / G2_BK;
  int soff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 8 * (4 * wid + j) + (lane >> 3);
    soff[j] = row * K + (((lane & 7) ^ g2_swz(row)) * 8);
  }
  const int l16 = lane & 15, lq = lane >> 4;
  for (;;) {
    const int tile = grab_unit(q, table, mode, me, xcc, s_slot, (u32)ntiles);
    if (tile < 0) break;
    int tm = tile / tiles_n, tn = tile % tiles_n;
    if ((mode & kGemmBlock2D) && (tiles_m & 3) == 0 && (tiles_n & 1) == 0 && ntiles % kXcds == 0) {
      const int bm = tiles_m / 4, bn = tiles_n / 2, g = tile % kXcds, jj = tile / kXcds;
      tm = (g >> 1) * bm + jj / bn;
      tn = (g & 1) * bn + jj % bn;
    }
    const u16* Ab = A + (size_t)tm * G2_BM * K;
    const u16* Bb = Bt + (size_t)tn * G2_BM * K;
    // glds n (0..15) of K-tile t: operand n >> 3, half (n >> 2) & 1, chunk n & 3
    auto glds_n = [&](int t, int n) {
      const int kind = n >> 3, h = (n >> 2) & 1, j = n & 3;
      const u16* src = (kind ? Bb : Ab) + (size_t)h * 128 * K + t * G2_BK;
      lds_t* dst = lds + (t & 1) * kG2Buf + (kind * 2 + h) * kG2Half + wid * 4096;
      glds16(src + soff[j], dst + j * 1024);
    };
    auto fp = [&](int b, int kind, int h, int r0, int s) -> const lds_t* {
      const int r = r0 + l16;
      return lds + b * kG2Buf + (kind * 2 + h) * kG2Half + r * 128 + (((4 * s + lq) ^ g2_swz(r)) << 4);
    };
    // read n (0..15) of substep s from buffer b: B blocks 0..7, then A blocks 0..7
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    bf16x8 xa[8], xb[8], ya[8], yb[8];

#pragma unroll
    for (int n = 0; n < 16; ++n) glds_n(0, n);
    if (nt > 1) {
#pragma unroll
      for (int n = 0; n < 16; ++n) glds_n(1, n);
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) GPBS_DSR(xb[j], fp(0, 1, wc, j * 16, 0));
#pragma unroll
    for (int i = 0; i < 8; ++i) GPBS_DSR(xa[i], fp(0, 0, wr, i * 16, 0));
    __builtin_amdgcn_sched_barrier(0);

    // one K-tile; PH 2: stage t+2 and read (t+1, 0), PH 1: read only, PH 0: last tile
    auto ktile = [&](int t, auto ph) {
      constexpr int PH = decltype(ph)::value;
      const int b = t & 1;
      // ---- M1: X; reads of (t, 1) -> Y
      GPBS_LGKM(0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < 64; ++k) {
        w4_mfma<1>(acc[k >> 3][k & 7], xb[k & 7], xa[k >> 3]);
        if ((k & 1) == 0 && k < 32) {
          const int n = k >> 1;
          if (n < 8) GPBS_DSR(yb[n], fp(b, 1, wc, n * 16, 1));
          else GPBS_DSR(ya[n - 8], fp(b, 0, wr, (n - 8) * 16, 1));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      GPBS_LGKM(0);
      if constexpr (PH > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- M2: Y; stage tile t+2 -> buffer b; reads of (t+1, 0) -> X
#pragma unroll
      for (int k = 0; k < 64; ++k) {
        w4_mfma<1>(acc[k >> 3][k & 7], yb[k & 7], ya[k >> 3]);
        if (k < 32) {
          const int n = k >> 1;
          if (k & 1) {
            if constexpr (PH == 2) glds_n(t + 2, n);
          } else if constexpr (PH > 0) {
            if (n < 8) GPBS_DSR(xb[n], fp(b ^ 1, 1, wc, n * 16, 0));
            else GPBS_DSR(xa[n - 8], fp(b ^ 1, 0, wr, (n - 8) * 16, 0));
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    int t = 0;
    for (; t + 2 < nt; ++t) ktile(t, std::integral_constant<int, 2>());
    if (t + 1 < nt) ktile(t++, std::integral_constant<int, 1>());
    ktile(t, std::integral_constant<int, 0>());
    // XDL results of the last MFMAs before the epilogue reads them
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
                 : "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]), "+a"(acc[7][4]),
                   "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7]));
    asm volatile(""
                 : "+a"(acc[6][0]), "+a"(acc[6][1]), "+a"(acc[6][2]), "+a"(acc[6][3]), "+a"(acc[6][4]),
                   "+a"(acc[6][5]), "+a"(acc[6][6]), "+a"(acc[6][7]));
    // C through LDS (every wave's reads retired before the last barrier;
    // no staging load in flight): 8-byte fragments at row m, chunk c8 ^ (m & 15)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = wr * 128 + i * 16 + l16;
        const int c8 = wc * 32 + j * 4 + lq;
        const u32 lo = (u32)f2bf(acc[i][j][0]) | ((u32)f2bf(acc[i][j][1]) << 16);
        const u32 hi = (u32)f2bf(acc[i][j][2]) | ((u32)f2bf(acc[i][j][3]) << 16);
        *(__attribute__((address_space(3))) u32x2*)(lds + m * 512 + ((c8 ^ (m & 15)) << 3)) = u32x2{lo, hi};
      }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 32; ++p) {
      const int row = p * 8 + (tid >> 5), c16 = tid & 31;
      u32x4 v = *(const __attribute__((address_space(3))) u32x4*)(lds + row * 512 + (((2 * c16) ^ (row & 14)) << 3));
      if (row & 1) v = u32x4{v.z, v.w, v.x, v.y};
      u32x4* dst = (u32x4*)(C + (size_t)(tm * G2_BM + row) * N + tn * G2_BM + c16 * 8);
      __builtin_nontemporal_store(v, dst);
    }
    __syncthreads();  // the next unit's prologue restages buffer 0
    count_unit(cnt, me, xcc, inst_per_tile, &t_last, refs_per_tile, miss_per_tile, q);
  }
  finish(q, status, (u32)ntiles);
}

// --------------- GEMM 256x256, 4 waves, row-split phases, 1.5-tile load lead ---
// PMC of k_gemm256w4i (profiles/r6/s56_gemm_pmc.txt): MFMA busy 0.49 with
// almost no LDS waits (0.017 of wave cycles) but SQ_WAIT_ANY 0.22 -- the
// mid-tile vmcnt(0) on tile t+1, whose loads had one K-tile of lead, against
// an L2 that misses a quarter of them.  The lead is set by when a buffer is
// free: w4i reads both K-substeps of every row from buffer t&1 until the
// middle of K-tile t.  Here a phase splits the wave's 128 rows instead:
//   M1(t): rows 0-63 of the wave tile (XA(t) x B(t), 64 MFMAs), reading
//          YA(t) = its A rows 64-127; M2(t): rows 64-127 (YA(t) x B(t)),
//          reading X(t+1) = XA(t+1) + B(t+1) into the other B register set.
// So once X(t) is read (barrier at the start of M1(t)), the B halves and the
// A rows 0-63 of buffer t&1 are free: part P0 of tile t+2 (B, A rows 0-63:
// 12 glds per wave) is staged during M1(t); part P1 (A rows 64-127, 4 glds)
// during M2(t), after the mid-tile barrier retires YA(t).  Both parts have
// 1.5 K-tiles to land: P0(t+1) is retired by vmcnt(16) before the mid-tile
// barrier of t (X(t+1) is read in M2(t)), P1(t) by vmcnt(16) before the
// barrier opening M1(t).  Fragments: XA, YA 32 VGPRs each, B 2 x 64.
// Host opts bit 22 (with bit 5).  Measured 1232 TF/s vs 1237 for w4i in the
// same process (profiles/r6/s57_kbench_w4j.jsonl): the longer lead buys
// nothing, so the load lead is not what holds the 4-wave kernels at ~0.49
// MFMA busy.  Not the default.
__global__ __launch_bounds__(G4_NT, 1) void k_gemm256w4j_bf16_tn(const u16* __restrict__ A,
                                                                const u16* __restrict__ Bt, u16* __restrict__ C,
                                                                int M, int N, int K, WorkQueue* q,
                                                                const PartTable* table, u32 mode, u32 me, u64* cnt,
                                                                u32 inst_per_tile, u32 refs_per_tile,
                                                                u32 miss_per_tile, u32* status) {
  __shared__ __attribute__((aligned(16))) char smem[kG2Lds + 16];
  lds_t* lds = (lds_t*)smem;
  int* s_slot = (int*)(smem + kG2Lds);
  const u32 xcc = xcc_id();
  u64 t_last = __builtin_amdgcn_s_memtime();
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  const int wr = wu >> 1, wc = wu & 1;
  const int tiles_m = M / G2_BM, tiles_n = N / G2_BM, ntiles = tiles_m * tiles_n;
  const int nt = K / G2_BK;
  // 1 KiB glds chunk c of a half = rows 8c .. 8c+7: per-lane source offset
  auto goff = [&](int c) {
    const int row = 8 * c + (lane >> 3);
    return row * K + (((lane & 7) ^ g2_swz(row)) * 8);
  };
  // P0: A chunks (wu & 1) * 4 + j of half wu >> 1, B chunks 4 wu + j of both
  // halves; P1: A chunks 8 + (wu & 1) * 4 + j of half wu >> 1
  int oa0[4], ob[4], oa1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    oa0[j] = goff((wu & 1) * 4 + j);
    ob[j] = goff(4 * wu + j);
    oa1[j] = goff(8 + (wu & 1) * 4 + j);
  }
  const int l16 = lane & 15, lq = lane >> 4;
  // fragment address = lane base [buffer][substep][A|B] + an immediate (row
  // block r0 * 128; r0 a multiple of 16 leaves the swizzle (r >> 1) & 7 to the lane)
  u32 fb[2][2][2];
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int kind = 0; kind < 2; ++kind)
        fb[b][s2][kind] = (u32)(size_t)(lds + b * kG2Buf + (kind * 2 + (kind ? wc : wr)) * kG2Half + l16 * 128 +
                                        (((4 * s2 + lq) ^ ((l16 >> 1) & 7)) << 4));
  for (;;) {
    const int tile = grab_unit(q, table, mode, me, xcc, s_slot, (u32)ntiles);
    if (tile < 0) break;
    int tm = tile / tiles_n, tn = tile % tiles_n;
    if ((mode & kGemmBlock2D) && (tiles_m & 3) == 0 && (tiles_n & 1) == 0 && ntiles % kXcds == 0) {
      const int bm = tiles_m / 4, bn = tiles_n / 2, g = tile % kXcds, jj = tile / kXcds;
      tm = (g >> 1) * bm + jj / bn;
      tn = (g & 1) * bn + jj % bn;
    }
    const u16* Ab = A + (size_t)tm * G2_BM * K;
    const u16* Bb = Bt + (size_t)tn * G2_BM * K;
    // glds n of part P0 (n 0..11: A 0..3, B half 0 4..7, B half 1 8..11) or P1 (n 0..3)
    // (ts = the source K-tile, buffer t & 1; past the last tile the loop
    // restages tile nt - 1 into the free buffer, which nobody reads)
    auto g_p0 = [&](int t, int n) {
      const int ts = t < nt ? t : nt - 1;
      lds_t* base = lds + (t & 1) * kG2Buf;
      if (n < 4) {
        const int h = wu >> 1, c = (wu & 1) * 4 + n;
        glds16(Ab + (size_t)h * 128 * K + ts * G2_BK + oa0[n], base + h * kG2Half + c * 1024);
      } else {
        const int h = (n - 4) >> 2, j = n & 3;
        glds16(Bb + (size_t)h * 128 * K + ts * G2_BK + ob[j], base + (2 + h) * kG2Half + (4 * wu + j) * 1024);
      }
    };
    auto g_p1 = [&](int t, int n) {
      const int ts = t < nt ? t : nt - 1;
      const int h = wu >> 1, c = 8 + (wu & 1) * 4 + n;
      glds16(Ab + (size_t)h * 128 * K + ts * G2_BK + oa1[n], lds + (t & 1) * kG2Buf + h * kG2Half + c * 1024);
    };
    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    bf16x8 xa[4][2], ya[4][2], b0[8][2], b1[8][2];

    // prologue: tiles 0 and 1 (nt even, host), then X(0)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int n = 0; n < 12; ++n) g_p0(t, n);
#pragma unroll
      for (int n = 0; n < 4; ++n) g_p1(t, n);
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) W4J_DSR(b0[j][s2], fb[0][s2][1], (j * 16) * 128);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) W4J_DSR(xa[i][s2], fb[0][s2][0], (i * 16) * 128);
    __builtin_amdgcn_sched_barrier(0);

    // one K-tile: PH 2 stages tile t+2 and reads X(t+1); PH 1 reads only; PH 0 last
    auto ktile = [&](int t, auto ph, auto bq, bf16x8 (&bc)[8][2], bf16x8 (&bn)[8][2]) {
      constexpr int PH = decltype(ph)::value;
      constexpr int b = decltype(bq)::value;  // t & 1
      GPBS_LGKM(0);  // X(t) landed
      if constexpr (PH == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // P1(t)
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- M1: rows 0-63; read YA(t); stage P0(t+2)
#pragma unroll
      for (int k = 0; k < 64; ++k) {
        const int s2 = k >> 5, i = (k >> 3) & 3, j = k & 7;
        w4_mfma<1>(acc[i][j], bc[j][s2], xa[i][s2]);
        if (k < 16 && (k & 1) == 0) {
          const int n = k >> 1;
          W4J_DSR(ya[n >> 1][n & 1], fb[b][n & 1][0], (64 + (n >> 1) * 16) * 128);
        }
        if constexpr (PH == 2) {
          if ((k & 1) && k < 24) g_p0(t + 2, k >> 1);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      GPBS_LGKM(0);  // YA(t) landed
      if constexpr (PH == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // P0(t+1)
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- M2: rows 64-127; read X(t+1); stage P1(t+2)
#pragma unroll
      for (int k = 0; k < 64; ++k) {
        const int s2 = k >> 5, i = (k >> 3) & 3, j = k & 7;
        w4_mfma<1>(acc[4 + i][j], bc[j][s2], ya[i][s2]);
        if constexpr (PH > 0) {
          if (k < 48 && (k & 1) == 0) {
            const int n = k >> 1;  // 0..23: B blocks, then A blocks
            if (n < 16) W4J_DSR(bn[n >> 1][n & 1], fb[1 - b][n & 1][1], ((n >> 1) * 16) * 128);
            else W4J_DSR(xa[(n - 16) >> 1][n & 1], fb[1 - b][n & 1][0], (((n - 16) >> 1) * 16) * 128);
          }
        }
        if constexpr (PH == 2) {
          if ((k & 1) && k < 8) g_p1(t + 2, k >> 1);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    using P2 = std::integral_constant<int, 2>;
    using Q0 = std::integral_constant<int, 0>;
    using Q1 = std::integral_constant<int, 1>;
    // one loop body for every K-tile (nt even, host): the last two tiles
    // stage and read clamped copies instead of a tail with its own register
    // assignment (which spilled)
    for (int t = 0; t < nt; t += 2) {
      ktile(t, P2(), Q0(), b0, b1);
      ktile(t + 1, P2(), Q1(), b1, b0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
                 : "+a"(acc[7][0]), "+a"(acc[7][1]), "+a"(acc[7][2]), "+a"(acc[7][3]), "+a"(acc[7][4]),
                   "+a"(acc[7][5]), "+a"(acc[7][6]), "+a"(acc[7][7]));
    asm volatile(""
                 : "+a"(acc[6][0]), "+a"(acc[6][1]), "+a"(acc[6][2]), "+a"(acc[6][3]), "+a"(acc[6][4]),
                   "+a"(acc[6][5]), "+a"(acc[6][6]), "+a"(acc[6][7]));
    __syncthreads();  // every wave's last LDS reads retired before C overwrites the buffers
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = wr * 128 + i * 16 + l16;
        const int c8 = wc * 32 + j * 4 + lq;
        const u32 lo = (u32)f2bf(acc[i][j][0]) | ((u32)f2bf(acc[i][j][1]) << 16);
        const u32 hi = (u32)f2bf(acc[i][j][2]) | ((u32)f2bf(acc[i][j][3]) << 16);
        *(__attribute__((address_space(3))) u32x2*)(lds + m * 512 + ((c8 ^ (m & 15)) << 3)) = u32x2{lo, hi};
      }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 32; ++p) {
      const int row = p * 8 + (tid >> 5), c16 = tid & 31;
      u32x4 v = *(const __attribute__((address_space(3))) u32x4*)(lds + row * 512 + (((2 * c16) ^ (row & 14)) << 3));
      if (row & 1) v = u32x4{v.z, v.w, v.x, v.y};
      u32x4* dst = (u32x4*)(C + (size_t)(tm * G2_BM + row) * N + tn * G2_BM + c16 * 8);
      __builtin_nontemporal_store(v, dst);
    }
    __syncthreads();
    count_unit(cnt, me, xcc, inst_per_tile, &t_last, refs_per_tile, miss_per_tile, q);
  }
  finish(q, status, (u32)ntiles);
}
#undef GPBS_DSR
#undef W4J_DSR
#undef GPBS_TOUCH
#undef GPBS_LGKM

// ------------------------------------------------------------ HBM stream ---
// dst = src (float4 copy), 16 B per lane, 16 loads in flight per thread: one
// 256-thread workgroup per CU keeps 64 KiB of reads in flight (enough for
// HBM3E at ~2 us loaded latency) while occupying only one wave slot per SIMD,
// so a co-resident GEMM keeps its two waves/SIMD (VGPR budget 512/SIMD: GEMM
// 2x136 + stream 80 + reduce 64 + gemv 96 = 512 fits; the old 4 WG/CU grids did not).
constexpr int SNT = 256, SUNROLL = 16, RUNROLL = 6;

template <int U, bool NTS>
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
    for (u64 i = base + threadIdx.x; i < end; i += (u64)SNT * U) {
      f32x4 v[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const u64 idx = i + (u64)k * SNT;
        if (idx < end) v[k] = __builtin_nontemporal_load(src + idx);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const u64 idx = i + (u64)k * SNT;
        if (idx < end) {
          if constexpr (NTS)
            __builtin_nontemporal_store(v[k], dst + idx);
          else
            dst[idx] = v[k];
        }
      }
    }
    count_unit(cnt, me, xcc, inst, &t_last, 2 * lines, 2 * lines, q);
  }
  finish(q, status, nchunks);
}

// ------------------------------------------------- reduce-copy (all-reduce) -
// out = a + b on bf16 (the traffic shape of a ring all-reduce step: two reads
// and one write per element).  Used as the collective tenant on one GPU; on
// N > 1 GPUs the tenant issues RCCL all-reduce over xGMI instead.
// Variants (gpbs_hip_set_reduce_opts, swept by scripts/kbench.py): NT threads
// per workgroup, U 16-byte element pairs in flight per thread, non-temporal
// (streaming) loads / stores on or off.
template <int NT, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(NT) void k_reduce_bf16(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
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
    for (u64 i = base + threadIdx.x; i < end; i += (u64)NT * U) {
      u32x4 x[U], y[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const u64 idx = i + (u64)k * NT;
        if (idx < end) {
          if constexpr (NTL) {
            x[k] = __builtin_nontemporal_load(a + idx);
            y[k] = __builtin_nontemporal_load(b + idx);
          } else {
            x[k] = a[idx];
            y[k] = b[idx];
          }
        }
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const u64 idx = i + (u64)k * NT;
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
        if constexpr (NTS)
          __builtin_nontemporal_store(r, out + idx);
        else
          out[idx] = r;
      }
    }
    count_unit(cnt, me, xcc, inst, &t_last, 3 * lines, 3 * lines, q);
  }
  finish(q, status, nchunks);
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
  if (mode & GATE_WAVEPRIO) __builtin_amdgcn_s_setprio(3);
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
  finish(q, status, nchunks);
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

int gpbs_hip_set_gemm_opts(int opts) {
  const int old = g_gemm_opts;
  if (opts >= 0) g_gemm_opts = opts;
  return old;
}

// Diagnostic: the buffer the STAMP variant (opts bit 6) writes to (device
// memory, kStampWgs * 8 * kStampTiles * kStampSlots u32); returns its size in
// u32 words.
int gpbs_hip_set_gemm_dbg(void* buf) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_dbg), &buf, sizeof(buf)) != hipSuccess) return -5;
  return kStampWgs * 8 * kStampTiles * kStampSlots + kStampPhWgs * 4;
}

int gpbs_hip_gemm_units(int M, int N) {
  if (M % G2_BM == 0 && N % G2_BM == 0) return (M / G2_BM) * (N / G2_BM);
  return (M / GBM) * (N / GBN);
}

int gpbs_hip_gemm_bf16(const void* A, const void* Bt, void* C, int M, int N, int K, void* q, const void* table,
                       unsigned mode, unsigned me, void* cnt, void* status, int grid, hipStream_t s) {
  if (M % GBM || N % GBN || K % GBK || M <= 0 || N <= 0 || K <= 0) return -22;
  if (M % G2_BM == 0 && N % G2_BM == 0) {
    const int ntiles = (M / G2_BM) * (N / G2_BM);
    if (grid <= 0) grid = 256;  // one workgroup per CU
    if (grid > ntiles) grid = ntiles;
    const u32 inst = (u32)((G2_BM / 16) * (G2_BM / 16) * (K / 32) + (K / G2_BK) * 64 + 128);
    const u32 refs = (u32)(((u64)2 * G2_BM * K * 2) / 128);
    const u32 miss = (u32)((((u64)M + N) * K * 2 / 128) / ntiles + (u64)G2_BM * G2_BM * 2 / 128);
    const u32 m2 = mode | ((g_gemm_opts & 1) ? kGemmXRange : 0u) |
                   ((g_gemm_opts & 8) && ntiles % kXcds == 0 ? kGemmBlock2D : 0u) |
                   ((g_gemm_opts & (1 << 23)) && (mode & 3) == GATE_NONE && grid == ntiles ? kGemmStatic : 0u);
    if ((g_gemm_opts & 32) && (K / G2_BK) % 2 == 0) {  // 4-wave 128x128-per-wave variant (plain tile queue)
      if (g_gemm_opts & (1 << 22))
        hipLaunchKernelGGL(k_gemm256w4j_bf16_tn, dim3(grid), dim3(G4_NT), 0, s, (const u16*)A, (const u16*)Bt,
                           (u16*)C, M, N, K, (WorkQueue*)q, (const PartTable*)table, m2, me, (u64*)cnt, inst, refs,
                           miss, (u32*)status);
      else if (g_gemm_opts & (1 << 21))
        hipLaunchKernelGGL(k_gemm256w4i_bf16_tn, dim3(grid), dim3(G4_NT), 0, s, (const u16*)A, (const u16*)Bt,
                           (u16*)C, M, N, K, (WorkQueue*)q, (const PartTable*)table, m2, me, (u64*)cnt, inst, refs,
                           miss, (u32*)status);
      else
        hipLaunchKernelGGL((g_gemm_opts & (1 << 20)) ? k_gemm256w4_bf16_tn<1> : k_gemm256w4_bf16_tn<0>, dim3(grid),
                           dim3(G4_NT), 0, s, (const u16*)A, (const u16*)Bt, (u16*)C, M, N, K, (WorkQueue*)q,
                           (const PartTable*)table, mode, me, (u64*)cnt, inst, refs, miss, (u32*)status);
      return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    if (g_gemm_opts & 524288) {  // bit 19: bit 18's schedule, counted waits on asm fragment reads
      hipLaunchKernelGGL(k_gemm256p2_bf16_tn, dim3(grid), dim3(G2_NT), 0, s, (const u16*)A, (const u16*)Bt, (u16*)C,
                         M, N, K, (WorkQueue*)q, (const PartTable*)table, mode, me, (u64*)cnt, inst, refs, miss,
                         (u32*)status);
      return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    if (g_gemm_opts & 262144) {  // bit 18: one barrier per K-tile, pipelined fragments
      hipLaunchKernelGGL(k_gemm256p_bf16_tn, dim3(grid), dim3(G2_NT), 0, s, (const u16*)A, (const u16*)Bt, (u16*)C,
                         M, N, K, (WorkQueue*)q, (const PartTable*)table, mode, me, (u64*)cnt, inst, refs, miss,
                         (u32*)status);
      return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    if (g_gemm_opts & 256) {  // 2 phases per K-tile (4 barriers); bit 10: streaming C stores
      // bit 12: balanced staging; bit 13: each group stages its own A half (4 glds per read interval)
      const bool nt = g_gemm_opts & 1024, bal = g_gemm_opts & 4096, own = g_gemm_opts & 8192;
      const bool one = g_gemm_opts & 16384;  // bit 14: one phase per K-tile; bit 15 (with 13): 32x32x16 MFMAs; bit 16 (with 13): C staged through LDS; bit 17 (with 16): its stores non-temporal
      auto k2 = one ? ((g_gemm_opts & 64) ? k_gemm256s2_bf16_tn<1, 0, 3> : k_gemm256s2_bf16_tn<0, 0, 3>)
                : (g_gemm_opts & 64)
                    ? (own ? k_gemm256s2_bf16_tn<1, 0, 2>
                           : bal ? k_gemm256s2_bf16_tn<1, 0, 1>
                                 : (nt ? k_gemm256s2_bf16_tn<1, 1, 0> : k_gemm256s2_bf16_tn<1, 0, 0>))
                    : (own ? ((g_gemm_opts & 32768)   ? k_gemm256s2_bf16_tn<0, 0, 6>
                           : (g_gemm_opts & 65536) ? ((g_gemm_opts & 131072) ? k_gemm256s2_bf16_tn<0, 0, 8> : k_gemm256s2_bf16_tn<0, 0, 7>)
                                                   : k_gemm256s2_bf16_tn<0, 0, 2>)
                           : bal ? k_gemm256s2_bf16_tn<0, 0, 1>
                                 : (nt ? k_gemm256s2_bf16_tn<0, 1, 0> : k_gemm256s2_bf16_tn<0, 0, 0>));
      hipLaunchKernelGGL(k2, dim3(grid), dim3(G2_NT), 0, s, (const u16*)A, (const u16*)Bt, (u16*)C, M, N, K,
                         (WorkQueue*)q, (const PartTable*)table, m2, me, (u64*)cnt, inst, refs, miss,
                         (u32*)status);
      return hipGetLastError() == hipSuccess ? 0 : -5;
    }
    auto kern = (g_gemm_opts & 64)  ? k_gemm256_bf16_tn<2, 1>
                : (g_gemm_opts & 16)  ? k_gemm256_bf16_tn<3>
                : (g_gemm_opts & 4) ? k_gemm256_bf16_tn<2>
                : (g_gemm_opts & 2) ? k_gemm256_bf16_tn<1>
                                    : k_gemm256_bf16_tn<0>;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(G2_NT), 0, s, (const u16*)A, (const u16*)Bt, (u16*)C, M, N,
                       K, (WorkQueue*)q, (const PartTable*)table, m2, me, (u64*)cnt, inst, refs, miss, (u32*)status);
    return hipGetLastError() == hipSuccess ? 0 : -5;
  }
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

static int g_stream_opts = 0;

// bit 0: temporal stores; bit 1: 8 (not 16) loads in flight per thread.
int gpbs_hip_set_stream_opts(int opts) {
  const int old = g_stream_opts;
  if (opts >= 0) g_stream_opts = opts;
  return old;
}

int gpbs_hip_stream_copy(const void* src, void* dst, unsigned long long bytes, unsigned chunk_bytes, void* q,
                         const void* table, unsigned mode, unsigned me, void* cnt, void* status, int grid, hipStream_t s) {
  if (bytes % 16 || chunk_bytes % 16 || chunk_bytes == 0) return -22;
  if (grid <= 0) grid = 256;  // one workgroup per CU (see SUNROLL)
  using K = void (*)(const f32x4*, f32x4*, u64, u32, WorkQueue*, const PartTable*, u32, u32, u64*, u32*);
  static const K tab[4] = {k_stream_copy<SUNROLL, true>, k_stream_copy<SUNROLL, false>, k_stream_copy<8, true>,
                           k_stream_copy<8, false>};
  hipLaunchKernelGGL(tab[g_stream_opts & 3], dim3(grid), dim3(SNT), 0, s, (const f32x4*)src, (f32x4*)dst, bytes / 16,
                     chunk_bytes / 16, (WorkQueue*)q, (const PartTable*)table, mode, me, (u64*)cnt, (u32*)status);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Default: 6 pairs in flight, streaming (non-temporal) loads, TEMPORAL
// stores: 5.57-5.76 TB/s vs 5.02-5.13 with non-temporal stores and 5.84 for
// torch.add on the same box (profiles/kbench_r2.jsonl); unroll depth and
// 512-thread workgroups are within noise.
static int g_reduce_opts = 8;

// bits 0-1: in-flight pairs per thread 6 / 8 / 4 / 12; bit 2: temporal loads;
// bit 3: temporal stores; bit 4: 512-thread workgroups.  Returns the old value.
int gpbs_hip_set_reduce_opts(int opts) {
  const int old = g_reduce_opts;
  if (opts >= 0) g_reduce_opts = opts;
  return old;
}

int gpbs_hip_reduce_bf16(const void* a, const void* b, void* out, unsigned long long bytes, unsigned chunk_bytes,
                         void* q, const void* table, unsigned mode, unsigned me, void* cnt, void* status, int grid, hipStream_t s) {
  if (bytes % 16 || chunk_bytes % 16 || chunk_bytes == 0) return -22;
  if (grid <= 0) grid = 256;
  using K = void (*)(const u32x4*, const u32x4*, u32x4*, u64, u32, WorkQueue*, const PartTable*, u32, u32, u64*, u32*);
#define RV(NT, U) {k_reduce_bf16<NT, U, true, true>, k_reduce_bf16<NT, U, false, true>, \
                   k_reduce_bf16<NT, U, true, false>, k_reduce_bf16<NT, U, false, false>}
  static const K table256[4][4] = {RV(256, 6), RV(256, 8), RV(256, 4), RV(256, 12)};
  static const K table512[4][4] = {RV(512, 6), RV(512, 8), RV(512, 4), RV(512, 12)};
#undef RV
  const int o = g_reduce_opts;
  const int nt = (o & 16) ? 512 : 256;
  const K kern = ((o & 16) ? table512 : table256)[o & 3][((o >> 2) & 1) | (((o >> 3) & 1) << 1)];
  hipLaunchKernelGGL(kern, dim3(grid), dim3(nt), 0, s, (const u32x4*)a, (const u32x4*)b, (u32x4*)out,
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
