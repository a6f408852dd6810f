// fp8 (OCP e4m3fn) weight-streaming linear for the Llama inference tenant
// (BASELINE config #5: "Llama-3-8B inference ... (CDNA4 fp8 MFMA)").
//
// Decode is a skinny GEMM: Y[M, N] = X[M, K] . W[N, K]^T with M = batch (<= 64)
// and N, K in the thousands, so its cost is streaming W from HBM once.  Storing
// W as fp8 halves those bytes against bf16.  Both operands go through the gfx950
// fp8 MFMA (v_mfma_f32_16x16x32_fp8_fp8, OCP e4m3); the accumulation is fp32 and
// the per-row scales are applied in the epilogue:
//     Y[m, n] = (sum_k Xq[m, k] Wq[n, k]) * sx[m] * sw[n]
// with sx / sw the absmax / 448 of each activation / weight row
// (k_quant_rows_fp8 produces both: run over W once at load time, over X per call).
//
// Work shape (CDNA4, 64-wide waves): one workgroup per 16 output columns, 8 waves
// splitting K in 256-byte blocks.  Lane (r = l & 15, g = l >> 4) streams row
// n0 + r of W, 16 bytes at k = kb + 64u + 16g (u = 0..3), i.e. 64 contiguous bytes
// per row per u and 8 x 16 B loads in flight per lane.  The A fragment (X rows, from
// L2) uses the SAME lane -> k permutation, so each MFMA sums a consistent set of 32
// k's and the product is exact regardless of the hardware's in-fragment k order.
// The eight wave partials are reduced through LDS.
#include "common.hpp"

namespace gpbs_fp8 {

using namespace gpbs_hip;

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;
constexpr int kQuantThreads = 256;
constexpr float kE4M3Max = 448.0f;

__device__ __forceinline__ float bf_lo(u32 v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(u32 v) { return __uint_as_float(v & 0xffff0000u); }

__device__ __forceinline__ unsigned short f2bf(float f) {
  u32 u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even
  return (unsigned short)(u >> 16);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Per-row symmetric quantisation bf16 -> e4m3fn.  grid = rows, block = 256.
// x: rows x (k8 * 8) bf16, q: rows x (k8 * 8) fp8, scale[row] = absmax / 448.
__global__ __launch_bounds__(kQuantThreads) void k_quant_rows_fp8(const u32x4* __restrict__ x, u32x2* __restrict__ q,
                                                                float* __restrict__ scale, int k8) {
  __shared__ float red[kQuantThreads / 64];
  const size_t row = blockIdx.x;
  const u32x4* xr = x + row * k8;
  float m = 0.f;
  for (int i = threadIdx.x; i < k8; i += kQuantThreads) {
    const u32x4 v = xr[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) m = fmaxf(m, fmaxf(fabsf(bf_lo(v[e])), fabsf(bf_hi(v[e]))));
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  float amax = red[0];
#pragma unroll
  for (int w = 1; w < kQuantThreads / 64; ++w) amax = fmaxf(amax, red[w]);
  const float s = amax > 0.f ? amax / kE4M3Max : 1.f;
  const float inv = amax > 0.f ? kE4M3Max / amax : 1.f;
  if (threadIdx.x == 0) scale[row] = s;
  u32x2* qr = q + row * k8;
  for (int i = threadIdx.x; i < k8; i += kQuantThreads) {
    const u32x4 v = xr[i];
    u32x2 o;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float a = fminf(fmaxf(bf_lo(v[2 * h]) * inv, -kE4M3Max), kE4M3Max);
      const float b = fminf(fmaxf(bf_hi(v[2 * h]) * inv, -kE4M3Max), kE4M3Max);
      const float c = fminf(fmaxf(bf_lo(v[2 * h + 1]) * inv, -kE4M3Max), kE4M3Max);
      const float d = fminf(fmaxf(bf_hi(v[2 * h + 1]) * inv, -kE4M3Max), kE4M3Max);
      int p = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
      p = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, p, true);
      o[h] = (u32)p;
    }
    qr[i] = o;
  }
}

template <int NT = kQuantThreads>
__device__ __forceinline__ float block_max256(float m, float* red) {
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int w = 1; w < NT / 64; ++w) r = fmaxf(r, red[w]);
  return r;
}

constexpr int kSwigluThreads = 1024;

__device__ __forceinline__ u32x2 pack_fp8x8(const float* v, float inv) {
  u32x2 o;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float c[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) c[e] = fminf(fmaxf(v[4 * h + e] * inv, -kE4M3Max), kE4M3Max);
    int p = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
    o[h] = (u32)__builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], p, true);
  }
  return o;
}

__device__ __forceinline__ float silu(float v) { return v / (1.f + __expf(-v)); }

// RMSNorm fused with the fp8 row quantiser (the producer of the qkv / gate-up
// linears' input): one workgroup per row, the normalised row never touches HBM in bf16.
__global__ __launch_bounds__(kQuantThreads) void k_rmsnorm_quant_fp8(const u32x4* __restrict__ x,
                                                                   const u32x4* __restrict__ w, u32x2* __restrict__ q,
                                                                   float* __restrict__ scale, int dim8, float eps) {
  __shared__ float red[2][kQuantThreads / 64];
  const size_t row = blockIdx.x;
  const u32x4* xr = x + row * dim8;
  float ss = 0.f;
  for (int i = threadIdx.x; i < dim8; i += kQuantThreads) {
    const u32x4 v = xr[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) ss += bf_lo(v[e]) * bf_lo(v[e]) + bf_hi(v[e]) * bf_hi(v[e]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  if ((threadIdx.x & 63) == 0) red[0][threadIdx.x >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int k = 0; k < kQuantThreads / 64; ++k) tot += red[0][k];
  const float rs = rsqrtf(tot / (float)(dim8 * 8) + eps);
  float m = 0.f;
  for (int i = threadIdx.x; i < dim8; i += kQuantThreads) {
    const u32x4 v = xr[i], g = w[i];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      m = fmaxf(m, fmaxf(fabsf(bf_lo(v[e]) * rs * bf_lo(g[e])), fabsf(bf_hi(v[e]) * rs * bf_hi(g[e]))));
  }
  const float amax = block_max256(m, red[1]);
  const float inv = amax > 0.f ? kE4M3Max / amax : 1.f;
  if (threadIdx.x == 0) scale[row] = amax > 0.f ? amax / kE4M3Max : 1.f;
  u32x2* qr = q + row * dim8;
  for (int i = threadIdx.x; i < dim8; i += kQuantThreads) {
    const u32x4 v = xr[i], g = w[i];
    float f[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      f[2 * e] = bf_lo(v[e]) * rs * bf_lo(g[e]);
      f[2 * e + 1] = bf_hi(v[e]) * rs * bf_hi(g[e]);
    }
    qr[i] = pack_fp8x8(f, inv);
  }
}

// SwiGLU on the packed gate|up output [rows, 2F] fused with the fp8 row
// quantiser: y = silu(gu[:, :F]) * gu[:, F:], emitted as e4m3 + row scale.
__global__ __launch_bounds__(kSwigluThreads) void k_swiglu_quant_fp8(const u32x4* __restrict__ gu,
                                                                  u32x2* __restrict__ q, float* __restrict__ scale,
                                                                  int f8) {
  __shared__ float red[kSwigluThreads / 64];
  const size_t row = blockIdx.x;
  const u32x4* a = gu + row * 2 * f8;
  const u32x4* b = a + f8;
  float m = 0.f;
  for (int i = threadIdx.x; i < f8; i += kSwigluThreads) {
    const u32x4 va = a[i], vb = b[i];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      m = fmaxf(m, fmaxf(fabsf(silu(bf_lo(va[e])) * bf_lo(vb[e])), fabsf(silu(bf_hi(va[e])) * bf_hi(vb[e]))));
  }
  const float amax = block_max256<kSwigluThreads>(m, red);
  const float inv = amax > 0.f ? kE4M3Max / amax : 1.f;
  if (threadIdx.x == 0) scale[row] = amax > 0.f ? amax / kE4M3Max : 1.f;
  u32x2* qr = q + row * f8;
  for (int i = threadIdx.x; i < f8; i += kSwigluThreads) {
    const u32x4 va = a[i], vb = b[i];
    float f[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      f[2 * e] = silu(bf_lo(va[e])) * bf_lo(vb[e]);
      f[2 * e + 1] = silu(bf_hi(va[e])) * bf_hi(vb[e]);
    }
    qr[i] = pack_fp8x8(f, inv);
  }
}

__device__ __forceinline__ long lo64(u32x4 v) { return (long)(((u64)v[1] << 32) | v[0]); }
__device__ __forceinline__ long hi64(u32x4 v) { return (long)(((u64)v[3] << 32) | v[2]); }

// MT = number of 16-row M tiles (M <= 16 * MT).  K % 256 == 0, N % 16 == 0.
template <int MT, int WV, bool NT>
__global__ __launch_bounds__(WV * 64) void k_fp8_gemm_skinny(const unsigned char* __restrict__ xq,
                                                              const float* __restrict__ sx,
                                                              const unsigned char* __restrict__ wq,
                                                              const float* __restrict__ sw,
                                                              unsigned short* __restrict__ y,
                                                              const unsigned short* __restrict__ resid, int M, int N,
                                                              int K) {
  __shared__ f32x4 red[WV][MT][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int k16 = K >> 4;  // 16-byte units per row
  const int nkb = K >> 8;  // 256-byte blocks
  // W is pre-shuffled (Fp8Weight): for strip n0/16, block kb, step u, the 64 lanes'
  // 16-byte pieces are one contiguous 1 KiB run in lane order, so every load
  // instruction is a fully coalesced 1 KiB read.
  const u32x4* wrow = reinterpret_cast<const u32x4*>(wq) + (size_t)blockIdx.x * nkb * 256 + lane;
  const u32x4* xb = reinterpret_cast<const u32x4*>(xq);
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int kb = w; kb < nkb; kb += 2 * WV) {
    const bool two = kb + WV < nkb;
    u32x4 b0[4], b1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) b0[u] = NT ? __builtin_nontemporal_load(wrow + kb * 256 + u * 64) : wrow[kb * 256 + u * 64];
    if (two) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        b1[u] = NT ? __builtin_nontemporal_load(wrow + (kb + WV) * 256 + u * 64) : wrow[(kb + WV) * 256 + u * 64];
    }
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = t * 16 + r;
      const u32x4* xr = xb + (size_t)m * k16 + g;
      u32x4 a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = m < M ? xr[kb * 16 + u * 4] : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(lo64(a[u]), lo64(b0[u]), acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(hi64(a[u]), hi64(b0[u]), acc[t], 0, 0, 0);
      }
      if (two) {
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] = m < M ? xr[(kb + WV) * 16 + u * 4] : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(lo64(a[u]), lo64(b1[u]), acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(hi64(a[u]), hi64(b1[u]), acc[t], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < MT; ++t) red[w][t][lane] = acc[t];
  __syncthreads();
  // C/D map of 16x16 MFMA: col = lane & 15 (n), row = 4 * (lane >> 4) + i (m).
  for (int e = threadIdx.x; e < MT * 64; e += WV * 64) {
    const int t = e >> 6, l = e & 63;
    f32x4 s = red[0][t][l];
#pragma unroll
    for (int v = 1; v < WV; ++v) s += red[v][t][l];
    const int n = n0 + (l & 15);
    const float wsc = sw[n];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = t * 16 + 4 * (l >> 4) + i;
      if (m < M) {
        float v = s[i] * sx[m] * wsc;
        if (resid) v += __uint_as_float((u32)resid[(size_t)m * N + n] << 16);  // fused residual add
        y[(size_t)m * N + n] = f2bf(v);
      }
    }
  }
}

}  // namespace gpbs_fp8

using namespace gpbs_fp8;

// Launch variant (microbench knob): bit 0 = non-temporal W loads instead of
// plain cached ones, bit 1 = 4 waves per workgroup instead of 8.
static int g_fp8_opts = 0;

template <int WV, bool NT>
static void launch_fp8(const unsigned char* xp, const float* sx, const unsigned char* wp, const float* sw,
                       unsigned short* yp, const unsigned short* rp, int M, int N, int K, hipStream_t s) {
  const dim3 grid(N / 16), block(WV * 64);
  if (M <= 16)
    hipLaunchKernelGGL((k_fp8_gemm_skinny<1, WV, NT>), grid, block, 0, s, xp, sx, wp, sw, yp, rp, M, N, K);
  else if (M <= 32)
    hipLaunchKernelGGL((k_fp8_gemm_skinny<2, WV, NT>), grid, block, 0, s, xp, sx, wp, sw, yp, rp, M, N, K);
  else
    hipLaunchKernelGGL((k_fp8_gemm_skinny<4, WV, NT>), grid, block, 0, s, xp, sx, wp, sw, yp, rp, M, N, K);
}

extern "C" {

int gpbs_hip_quant_rows_fp8(const void* x, void* q, float* scale, int rows, int k, hipStream_t s) {
  if (rows <= 0 || k <= 0 || k % 8) return -22;
  hipLaunchKernelGGL(k_quant_rows_fp8, dim3(rows), dim3(kQuantThreads), 0, s, (const u32x4*)x, (u32x2*)q, scale,
                     k / 8);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_rmsnorm_quant_fp8(const void* x, const void* w, void* q, float* scale, int rows, int dim, float eps,
                               hipStream_t s) {
  if (rows <= 0 || dim <= 0 || dim % 8) return -22;
  hipLaunchKernelGGL(k_rmsnorm_quant_fp8, dim3(rows), dim3(kQuantThreads), 0, s, (const u32x4*)x, (const u32x4*)w,
                     (u32x2*)q, scale, dim / 8, eps);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_swiglu_quant_fp8(const void* gu, void* q, float* scale, int rows, int f, hipStream_t s) {
  if (rows <= 0 || f <= 0 || f % 8) return -22;
  hipLaunchKernelGGL(k_swiglu_quant_fp8, dim3(rows), dim3(kSwigluThreads), 0, s, (const u32x4*)gu, (u32x2*)q, scale,
                     f / 8);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_fp8_set_opts(int opts) {
  const int prev = g_fp8_opts;
  g_fp8_opts = opts;
  return prev;
}

int gpbs_hip_fp8_linear_res(const void* xq, const float* sx, const void* wq, const float* sw, void* y,
                            const void* resid, int M, int N, int K, hipStream_t s) {
  if (M <= 0 || M > 64 || N <= 0 || N % 16 || K <= 0 || K % 256) return -22;
  const auto* xp = (const unsigned char*)xq;
  const auto* wp = (const unsigned char*)wq;
  auto* yp = (unsigned short*)y;
  const auto* rp = (const unsigned short*)resid;
  switch (g_fp8_opts & 3) {
    case 0: launch_fp8<kWaves, false>(xp, sx, wp, sw, yp, rp, M, N, K, s); break;
    case 1: launch_fp8<kWaves, true>(xp, sx, wp, sw, yp, rp, M, N, K, s); break;
    case 2: launch_fp8<4, true>(xp, sx, wp, sw, yp, rp, M, N, K, s); break;
    default: launch_fp8<4, false>(xp, sx, wp, sw, yp, rp, M, N, K, s); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_fp8_linear(const void* xq, const float* sx, const void* wq, const float* sw, void* y, int M, int N, int K,
                        hipStream_t s) {
  return gpbs_hip_fp8_linear_res(xq, sx, wq, sw, y, nullptr, M, N, K, s);
}

}  // extern "C"
