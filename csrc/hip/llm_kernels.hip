// Fused elementwise kernels of the Llama-3 tenants (gfx950), bf16 in/out with
// fp32 arithmetic; 16-byte (8 x bf16) vector accesses throughout.
//   k_rmsnorm_bf16 : y = x * rsqrt(mean(x^2) + eps) * w, one workgroup per row
//                    (256 threads: wave reduction by shuffles, 4 partials in LDS)
//   k_swiglu_bf16  : y = silu(a) * b (the SwiGLU gate, fused so the 14336-wide
//                    intermediate is read once instead of three times)
//   k_rope_bf16    : rotary embedding on interleaved pairs, positions pos..pos+S-1
#include <algorithm>

#include "common.hpp"

namespace gpbs_hip {

__device__ __forceinline__ float bfl(u32 w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfh(u32 w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ u32 pack2(float lo, float hi) {
  return (u32)__builtin_bit_cast(u16, (__bf16)lo) | ((u32)__builtin_bit_cast(u16, (__bf16)hi) << 16);
}

constexpr int kNormThreads = 256;

__global__ __launch_bounds__(kNormThreads) void k_rmsnorm_bf16(const u32x4* __restrict__ x, const u32x4* __restrict__ w,
                                                              u32x4* __restrict__ y, int dim8, float eps) {
  __shared__ float part[kNormThreads / 64];
  const int row = blockIdx.x;
  const u32x4* xr = x + (size_t)row * dim8;
  u32x4* yr = y + (size_t)row * dim8;
  float ss = 0.f;
  for (int i = threadIdx.x; i < dim8; i += kNormThreads) {
    const u32x4 v = xr[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = bfl(v[e]), b = bfh(v[e]);
      ss += a * a + b * b;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int k = 0; k < kNormThreads / 64; ++k) tot += part[k];
  const float r = rsqrtf(tot / (float)(dim8 * 8) + eps);
  for (int i = threadIdx.x; i < dim8; i += kNormThreads) {
    const u32x4 v = xr[i], g = w[i];
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2(bfl(v[e]) * r * bfl(g[e]), bfh(v[e]) * r * bfh(g[e]));
    yr[i] = o;
  }
}

__device__ __forceinline__ float silu(float v) { return v / (1.f + __expf(-v)); }

__global__ __launch_bounds__(256) void k_swiglu_bf16(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                    u32x4* __restrict__ y, size_t n8) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    const u32x4 va = a[i], vb = b[i];
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2(silu(bfl(va[e])) * bfl(vb[e]), silu(bfh(va[e])) * bfh(vb[e]));
    y[i] = o;
  }
}

// x, y: [B][S][H][hd] bf16 contiguous; cos/sin: [max_seq][hd/2] fp32.
// Each thread rotates 4 interleaved pairs (16 B).
__global__ __launch_bounds__(256) void k_rope_bf16(const u32x4* __restrict__ x, u32x4* __restrict__ y,
                                                  const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                  int S, int H, int hd, int pos, const int* __restrict__ dpos,
                                                  size_t n8) {
  if (dpos) pos += *dpos;  // device-resident position (graph-captured decode)
  const int per_head = hd / 8;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % per_head);                 // 8-element chunk within the head
    const int s = (int)((i / per_head / H) % S);       // sequence index
    const float* cr = cosb + (size_t)(pos + s) * (hd / 2) + c * 4;
    const float* sr = sinb + (size_t)(pos + s) * (hd / 2) + c * 4;
    const u32x4 v = x[i];
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = bfl(v[e]), b = bfh(v[e]), cs = cr[e], sn = sr[e];
      o[e] = pack2(a * cs - b * sn, a * sn + b * cs);
    }
    y[i] = o;
  }
}

}  // namespace gpbs_hip

using namespace gpbs_hip;

extern "C" {

int gpbs_hip_rmsnorm_bf16(const void* x, const void* w, void* y, int rows, int dim, float eps, hipStream_t s) {
  if (rows <= 0 || dim <= 0 || dim % 8) return -22;
  hipLaunchKernelGGL(k_rmsnorm_bf16, dim3(rows), dim3(kNormThreads), 0, s, (const u32x4*)x, (const u32x4*)w,
                     (u32x4*)y, dim / 8, eps);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_swiglu_bf16(const void* a, const void* b, void* y, unsigned long long n, hipStream_t s) {
  if (n % 8) return -22;
  const size_t n8 = n / 8;
  int grid = (int)std::min<size_t>((n8 + 255) / 256, 256 * 8);
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_swiglu_bf16, dim3(grid), dim3(256), 0, s, (const u32x4*)a, (const u32x4*)b, (u32x4*)y, n8);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_rope_bf16(const void* x, void* y, const float* cosb, const float* sinb, int B, int S, int H, int hd,
                       int pos, hipStream_t s) {
  if (hd % 8 || B <= 0 || S <= 0 || H <= 0) return -22;
  const size_t n8 = (size_t)B * S * H * hd / 8;
  int grid = (int)std::min<size_t>((n8 + 255) / 256, 256 * 8);
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_rope_bf16, dim3(grid), dim3(256), 0, s, (const u32x4*)x, (u32x4*)y, cosb, sinb, S, H, hd, pos,
                     (const int*)nullptr, n8);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Same, with the start position read from device memory at run time (int32), so
// a captured HIP graph replays at the current position.
int gpbs_hip_rope_bf16_dpos(const void* x, void* y, const float* cosb, const float* sinb, int B, int S, int H, int hd,
                            const int* dpos, hipStream_t s) {
  if (hd % 8 || B <= 0 || S <= 0 || H <= 0 || !dpos) return -22;
  const size_t n8 = (size_t)B * S * H * hd / 8;
  int grid = (int)std::min<size_t>((n8 + 255) / 256, 256 * 8);
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_rope_bf16, dim3(grid), dim3(256), 0, s, (const u32x4*)x, (u32x4*)y, cosb, sinb, S, H, hd, 0,
                     dpos, n8);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // extern "C"
