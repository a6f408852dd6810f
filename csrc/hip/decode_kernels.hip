// Fused single-token decode kernels for the graph-captured Llama decode step
// (config #5).  Every launch saved is ~4-5 us per layer at batch 8, so the
// attention block runs in two launches after the qkv linear:
//
//   k_qkv_rope_cache : packed qkv linear output [B, (H + 2 Hkv) hd] ->
//                      q with RoPE -> q_out [B, H, hd]; k with RoPE and v written
//                      straight into the static KV cache [B, Hkv, C, hd] at the
//                      device-resident position (replaces 2 slice copies, 2 RoPE
//                      launches, 2 index_copy_ and their transposes)
//   k_decode_attn    : grouped-query attention of the new token over cache rows
//                      0..pos: one workgroup per (batch, KV head), the G query
//                      heads of the group share every K/V row read; 4 waves split
//                      the keys (a lane owns a key for QK^T, a lane owns 2 dims
//                      for PV), online softmax, wave partials merged in LDS.
#include <algorithm>

#include "common.hpp"

namespace gpbs_dec {

using namespace gpbs_hip;

__device__ __forceinline__ float bfl(u32 w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfh(u32 w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ u32 pack2(float lo, float hi) {
  return (u32)__builtin_bit_cast(u16, (__bf16)lo) | ((u32)__builtin_bit_cast(u16, (__bf16)hi) << 16);
}

__global__ __launch_bounds__(256) void k_qkv_rope_cache(const u32x4* __restrict__ qkv, const float* __restrict__ cosb,
                                                        const float* __restrict__ sinb, const int* __restrict__ dpos,
                                                        u32x4* __restrict__ qo, u32x4* __restrict__ kc,
                                                        u32x4* __restrict__ vc, int B, int H, int Hkv, int C, int hd) {
  const int pos = *dpos;
  const int per_head = hd / 8, heads = H + 2 * Hkv;
  const size_t n8 = (size_t)B * heads * per_head;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % per_head);
    const int hh = (int)((i / per_head) % heads);
    const int b = (int)(i / per_head / heads);
    const u32x4 v = qkv[i];
    if (hh >= H + Hkv) {  // v: plain copy into the cache row
      vc[(((size_t)b * Hkv + (hh - H - Hkv)) * C + pos) * per_head + c] = v;
      continue;
    }
    const float* cr = cosb + (size_t)pos * (hd / 2) + c * 4;
    const float* sr = sinb + (size_t)pos * (hd / 2) + c * 4;
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float a = bfl(v[e]), bb = bfh(v[e]), cs = cr[e], sn = sr[e];
      o[e] = pack2(a * cs - bb * sn, a * sn + bb * cs);
    }
    if (hh < H)
      qo[((size_t)b * H + hh) * per_head + c] = o;
    else
      kc[(((size_t)b * Hkv + (hh - H)) * C + pos) * per_head + c] = o;
  }
}

constexpr int kHd = 128;  // head_dim of every Llama-3 size
constexpr int kAttnWaves = 8;

__device__ __forceinline__ float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// q [B, H, 128], caches [B, Hkv, C, 128], out [B, H * 128]; H = G * Hkv.
template <int G>
__global__ __launch_bounds__(kAttnWaves * 64) void k_decode_attn(const u32x4* __restrict__ q,
                                                               const u32x4* __restrict__ kc,
                                                               const u32* __restrict__ vc,
                                                               const int* __restrict__ dpos, u32* __restrict__ out,
                                                               float* __restrict__ ws, int Hkv, int C, float scale,
                                                               int nsplit) {
  __shared__ float qs[G][kHd];
  __shared__ float ms[kAttnWaves][G], ls[kAttnWaves][G];
  __shared__ float os[kAttnWaves][G][kHd];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int split = blockIdx.x % nsplit, bh = blockIdx.x / nsplit;
  const int b = bh / Hkv, kvh = bh % Hkv;
  const int L = min(*dpos + 1, C);  // keys 0..pos
  // flash-decoding split: this workgroup takes keys [k0, k1) (64-aligned chunks)
  const int chunk = ((L + nsplit - 1) / nsplit + 63) & ~63;
  const int k0 = split * chunk, k1 = min(L, k0 + chunk);
  const int H = G * Hkv;
  // stage the group's queries (pre-scaled) in LDS: read as broadcasts below
  for (int e = threadIdx.x; e < G * kHd / 8; e += kAttnWaves * 64) {
    const int g = e / (kHd / 8), c = e % (kHd / 8);
    const u32x4 v = q[((size_t)b * H + kvh * G + g) * (kHd / 8) + c];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      qs[g][c * 8 + 2 * k] = bfl(v[k]) * scale;
      qs[g][c * 8 + 2 * k + 1] = bfh(v[k]) * scale;
    }
  }
  __syncthreads();
  const size_t head = (size_t)b * Hkv + kvh;
  const u32x4* kh = kc + head * C * (kHd / 8);
  const u32* vh = vc + head * C * (kHd / 2);
  // PV lane map: key group kg = lane >> 4 takes keys kg, kg + 4, ...; dl = lane & 15
  // owns dims 8 dl .. 8 dl + 7 (one 16-byte V load per key)
  const int kg = lane >> 4, dl = lane & 15;
  float m[G], l[G], o[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY, l[g] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[g][e] = 0.f;
  }

  for (int base = k0 + w * 64; base < k1; base += kAttnWaves * 64) {
    const int j = base + lane;
    float s[G];
#pragma unroll
    for (int g = 0; g < G; ++g) s[g] = 0.f;
    // opaque zero: keeps the (loop-invariant) LDS query reads inside this loop, so
    // the compiler does not hoist G x 128 floats into registers and spill
    int z = 0;
    asm volatile("" : "+s"(z));
    const float* qz = &qs[0][0] + z;
    if (j < k1) {
      const u32x4* kr = kh + (size_t)j * (kHd / 8);
      u32x4 krow[kHd / 8];  // the lane's whole 256-byte key row in flight at once
#pragma unroll
      for (int c = 0; c < kHd / 8; ++c) krow[c] = kr[c];
#pragma unroll
      for (int c = 0; c < kHd / 8; ++c) {
        const u32x4 kv = krow[c];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float k0 = bfl(kv[k]), k1 = bfh(kv[k]);
#pragma unroll
          for (int g = 0; g < G; ++g) s[g] += qz[g * kHd + c * 8 + 2 * k] * k0 + qz[g * kHd + c * 8 + 2 * k + 1] * k1;
        }
      }
    }
    const int nk = min(64, k1 - base);
    float p[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float sg = j < k1 ? s[g] : -INFINITY;
      const float mn = fmaxf(m[g], wmax(sg));
      const float corr = __expf(m[g] - mn);
      p[g] = j < k1 ? __expf(sg - mn) : 0.f;
      l[g] = l[g] * corr + wsum(p[g]);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[g][e] *= corr;
      m[g] = mn;
    }
    // PV: 16 rounds of 4 keys (one per key group), 16-byte V loads, weights by shuffle
    const u32x4* vb = reinterpret_cast<const u32x4*>(vh) + (size_t)base * (kHd / 8) + dl;
#pragma unroll 4
    for (int t = 0; t < 16; ++t) {
      const int jj = 4 * t + kg;
      float pj[G];
#pragma unroll
      for (int g = 0; g < G; ++g) pj[g] = __shfl(p[g], jj, 64);
      if (jj < nk) {
        const u32x4 vv = vb[(size_t)jj * (kHd / 8)];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v0 = bfl(vv[e]), v1 = bfh(vv[e]);
#pragma unroll
          for (int g = 0; g < G; ++g) {
            o[g][2 * e] += pj[g] * v0;
            o[g][2 * e + 1] += pj[g] * v1;
          }
        }
      }
    }
  }
  // sum the 4 key groups' partials (lanes dl, dl + 16, dl + 32, dl + 48)
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[g][e] += __shfl_xor(o[g][e], 16, 64);
      o[g][e] += __shfl_xor(o[g][e], 32, 64);
    }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (kg == 0)
#pragma unroll
      for (int e = 0; e < 8; ++e) os[w][g][8 * dl + e] = o[g][e];
    if (lane == 0) ms[w][g] = m[g], ls[w][g] = l[g];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < G * 64; e += kAttnWaves * 64) {
    const int g = e / 64, d = 2 * (e % 64);
    float M = -INFINITY;
#pragma unroll
    for (int v = 0; v < kAttnWaves; ++v) M = fmaxf(M, ms[v][g]);
    float Ls = 0.f, a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int v = 0; v < kAttnWaves; ++v) {
      const float f = ms[v][g] == -INFINITY ? 0.f : __expf(ms[v][g] - M);
      Ls += ls[v][g] * f;
      a0 += os[v][g][d] * f;
      a1 += os[v][g][d + 1] * f;
    }
    if (nsplit == 1) {
      const float inv = 1.f / Ls;
      out[((size_t)b * H + kvh * G + g) * (kHd / 2) + d / 2] = pack2(a0 * inv, a1 * inv);
    } else {  // partial (max, sum, unnormalised o) for k_decode_attn_combine
      float* p = ws + ((size_t)blockIdx.x * G + g) * (kHd + 2);
      p[d] = a0;
      p[d + 1] = a1;
      if (d == 0) p[kHd] = M, p[kHd + 1] = Ls;
    }
  }
}

// Merge the nsplit partials of each (batch, KV head): grid B * Hkv, G * 64 threads.
__global__ __launch_bounds__(512) void k_decode_attn_combine(const float* __restrict__ ws, u32* __restrict__ out,
                                                             int Hkv, int G, int nsplit) {
  const int bh = blockIdx.x, b = bh / Hkv, kvh = bh % Hkv;
  const int g = threadIdx.x / 64, d = 2 * (threadIdx.x % 64);
  if (g >= G) return;
  float M = -INFINITY;
  for (int sp = 0; sp < nsplit; ++sp) M = fmaxf(M, ws[(((size_t)bh * nsplit + sp) * G + g) * (kHd + 2) + kHd]);
  float Ls = 0.f, a0 = 0.f, a1 = 0.f;
  for (int sp = 0; sp < nsplit; ++sp) {
    const float* p = ws + (((size_t)bh * nsplit + sp) * G + g) * (kHd + 2);
    const float f = p[kHd] == -INFINITY ? 0.f : __expf(p[kHd] - M);
    Ls += p[kHd + 1] * f;
    a0 += p[d] * f;
    a1 += p[d + 1] * f;
  }
  const float inv = 1.f / Ls;
  out[((size_t)b * Hkv * G + kvh * G + g) * (kHd / 2) + d / 2] = pack2(a0 * inv, a1 * inv);
}

}  // namespace gpbs_dec

using namespace gpbs_dec;

extern "C" {

int gpbs_hip_qkv_rope_cache(const void* qkv, const float* cosb, const float* sinb, const int* dpos, void* qo, void* kc,
                            void* vc, int B, int H, int Hkv, int C, int hd, hipStream_t s) {
  if (B <= 0 || H <= 0 || Hkv <= 0 || C <= 0 || hd % 8 || !dpos) return -22;
  const size_t n8 = (size_t)B * (H + 2 * Hkv) * hd / 8;
  int grid = (int)std::min<size_t>((n8 + 255) / 256, 2048);
  hipLaunchKernelGGL(k_qkv_rope_cache, dim3(grid), dim3(256), 0, s, (const u32x4*)qkv, cosb, sinb, dpos, (u32x4*)qo,
                     (u32x4*)kc, (u32x4*)vc, B, H, Hkv, C, hd);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int gpbs_hip_decode_attn(const void* q, const void* kc, const void* vc, const int* dpos, void* out, void* ws,
                         int nsplit, int B, int H, int Hkv, int C, int hd, float scale, hipStream_t s) {
  if (hd != kHd || B <= 0 || Hkv <= 0 || H % Hkv || C <= 0 || !dpos || nsplit < 1 || (nsplit > 1 && !ws)) return -22;
  const int G = H / Hkv;
  const dim3 grid(B * Hkv * nsplit), block(kAttnWaves * 64);
  float* w = (float*)ws;
  switch (G) {
    case 1: hipLaunchKernelGGL(k_decode_attn<1>, grid, block, 0, s, (const u32x4*)q, (const u32x4*)kc, (const u32*)vc,
                               dpos, (u32*)out, w, Hkv, C, scale, nsplit); break;
    case 2: hipLaunchKernelGGL(k_decode_attn<2>, grid, block, 0, s, (const u32x4*)q, (const u32x4*)kc, (const u32*)vc,
                               dpos, (u32*)out, w, Hkv, C, scale, nsplit); break;
    case 4: hipLaunchKernelGGL(k_decode_attn<4>, grid, block, 0, s, (const u32x4*)q, (const u32x4*)kc, (const u32*)vc,
                               dpos, (u32*)out, w, Hkv, C, scale, nsplit); break;
    case 8: hipLaunchKernelGGL(k_decode_attn<8>, grid, block, 0, s, (const u32x4*)q, (const u32x4*)kc, (const u32*)vc,
                               dpos, (u32*)out, w, Hkv, C, scale, nsplit); break;
    default: return -22;
  }
  if (nsplit > 1)
    hipLaunchKernelGGL(k_decode_attn_combine, dim3(B * Hkv), dim3(G * 64), 0, s, (const float*)w, (u32*)out, Hkv, G,
                       nsplit);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

}  // extern "C"
