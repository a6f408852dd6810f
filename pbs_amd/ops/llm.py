"""Torch-facing wrappers of the Llama tenant kernels (csrc/hip/llm_kernels.hip).

Inference-only (no autograd): the decode path of ``LlamaDecoder``.  The
library must load on a GPU box -- shape/dtype violations raise instead of
falling back to eager PyTorch.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from .kernels import _check, _ptr, _stream, lib


def _need(t: torch.Tensor, what: str):
    if not (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous()):
        raise ValueError(f"{what}: need a contiguous bf16 CUDA tensor, got {t.dtype} {t.device} "
                         f"contiguous={t.is_contiguous()}")


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    """y = x * rsqrt(mean(x^2, -1) + eps) * w (fp32 statistics)."""
    x = x.contiguous()
    _need(x, "rmsnorm x")
    w = w.to(torch.bfloat16).contiguous()
    dim = x.shape[-1]
    if w.numel() != dim or dim % 8:
        raise ValueError(f"rmsnorm: weight {tuple(w.shape)} vs dim {dim} (dim % 8 == 0 required)")
    y = torch.empty_like(x)
    _check(lib().gpbs_hip_rmsnorm_bf16(_ptr(x), _ptr(w), _ptr(y), x.numel() // dim, dim, C.c_float(eps),
                                       _stream()), "rmsnorm_bf16")
    return y


def swiglu(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """y = silu(a) * b."""
    a, b = a.contiguous(), b.contiguous()
    _need(a, "swiglu a")
    _need(b, "swiglu b")
    if a.shape != b.shape or a.numel() % 8:
        raise ValueError(f"swiglu: shapes {tuple(a.shape)} / {tuple(b.shape)}")
    y = torch.empty_like(a)
    _check(lib().gpbs_hip_swiglu_bf16(_ptr(a), _ptr(b), _ptr(y), a.numel(), _stream()), "swiglu_bf16")
    return y


def rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos: int) -> torch.Tensor:
    """Rotary embedding on interleaved pairs; x [B, S, H, hd], cos/sin fp32
    [max_seq, hd/2]; token s gets angle row pos + s."""
    x = x.contiguous()
    _need(x, "rope x")
    B, S, H, hd = x.shape
    if cos.dtype != torch.float32 or cos.shape[-1] * 2 != hd or pos + S > cos.shape[0]:
        raise ValueError(f"rope: tables {tuple(cos.shape)} {cos.dtype} for hd={hd}, pos={pos}, S={S}")
    y = torch.empty_like(x)
    _check(lib().gpbs_hip_rope_bf16(_ptr(x), _ptr(y), _ptr(cos.contiguous()), _ptr(sin.contiguous()), B, S, H, hd,
                                    int(pos), _stream()), "rope_bf16")
    return y



def rope_dpos(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos_t: torch.Tensor) -> torch.Tensor:
    """rope() with the start position in a 1-element int32 CUDA tensor (read by
    the kernel at run time: valid inside a captured graph).  No bounds check on
    the device value: the caller keeps pos + S <= cos.shape[0]."""
    x = x.contiguous()
    _need(x, "rope x")
    B, S, H, hd = x.shape
    if cos.dtype != torch.float32 or cos.shape[-1] * 2 != hd or pos_t.dtype != torch.int32 or not pos_t.is_cuda:
        raise ValueError(f"rope_dpos: tables {tuple(cos.shape)} {cos.dtype}, pos {pos_t.dtype} {pos_t.device}")
    y = torch.empty_like(x)
    _check(lib().gpbs_hip_rope_bf16_dpos(_ptr(x), _ptr(y), _ptr(cos), _ptr(sin), B, S, H, hd, _ptr(pos_t),
                                         _stream()), "rope_bf16_dpos")
    return y


def qkv_rope_cache(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, pos_t: torch.Tensor, kc: torch.Tensor,
                   vc: torch.Tensor, n_heads: int) -> torch.Tensor:
    """One-token decode: split the packed qkv [B, 1, (H + 2 Hkv) hd], RoPE q and k
    at the device position pos_t (int32 [1]), write k / v into the caches
    [B, Hkv, C, hd] at that row, return q [B, H, hd]."""
    B, Hkv, Cn, hd = kc.shape
    _need(qkv, "qkv_rope_cache qkv")
    _need(kc, "qkv_rope_cache kc")
    _need(vc, "qkv_rope_cache vc")
    if qkv.numel() != B * (n_heads + 2 * Hkv) * hd or vc.shape != kc.shape or cos.shape[-1] * 2 != hd \
            or pos_t.dtype != torch.int32:
        raise ValueError(f"qkv_rope_cache: qkv {tuple(qkv.shape)} vs cache {tuple(kc.shape)}, H={n_heads}")
    # the kernel indexes the RoPE tables and the cache rows with the device
    # position: the tables must cover every cache row, dtypes as it assumes
    if cos.shape[0] < Cn or sin.shape != cos.shape or cos.dtype != torch.float32 or sin.dtype != torch.float32 \
            or kc.dtype != torch.bfloat16 or vc.dtype != torch.bfloat16 or qkv.dtype != torch.bfloat16:
        raise ValueError(f"qkv_rope_cache: rope tables {tuple(cos.shape)} {cos.dtype} must cover {Cn} cache rows "
                         f"(fp32), caches/qkv bf16")
    q = torch.empty(B, n_heads, hd, dtype=torch.bfloat16, device=qkv.device)
    _check(lib().gpbs_hip_qkv_rope_cache(_ptr(qkv), _ptr(cos), _ptr(sin), _ptr(pos_t), _ptr(q), _ptr(kc), _ptr(vc),
                                         B, n_heads, Hkv, Cn, hd, _stream()), "qkv_rope_cache")
    return q


def decode_attn(q: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, pos_t: torch.Tensor,
                nsplit: Optional[int] = None) -> torch.Tensor:
    """Grouped-query attention of one new token per sequence over cache rows
    0..pos (pos_t int32 [1] on device): q [B, H, 128] -> [B, H * 128].  The keys
    are split over `nsplit` workgroups per (batch, KV head) (flash-decoding,
    default: enough to give the chip >= 256 workgroups) and merged by a combine
    kernel."""
    B, Hkv, Cn, hd = kc.shape
    H = q.shape[1]
    _need(q, "decode_attn q")
    if hd != 128 or H % Hkv or (H // Hkv) not in (1, 2, 4, 8) or q.shape != (B, H, hd):
        raise ValueError(f"decode_attn: q {tuple(q.shape)}, cache {tuple(kc.shape)} (head_dim 128, G in 1/2/4/8)")
    out = torch.empty(B, H * hd, dtype=torch.bfloat16, device=q.device)
    if nsplit is None:
        nsplit = max(1, min(8, -(-256 // (B * Hkv)), -(-Cn // 64)))
    ws = torch.empty(B * Hkv * nsplit * (H // Hkv) * (hd + 2), dtype=torch.float32, device=q.device) \
        if nsplit > 1 else None
    _check(lib().gpbs_hip_decode_attn(_ptr(q), _ptr(kc), _ptr(vc), _ptr(pos_t), _ptr(out), _ptr(ws), nsplit, B, H,
                                      Hkv, Cn, hd, C.c_float(hd ** -0.5), _stream()), "decode_attn")
    return out

# --------------------------------------------------------------------------- fp8 (config #5, CDNA4 fp8 MFMA)
FP8_MAX = 448.0  # OCP e4m3fn (gfx950), not the MI300 fnuz variant
FP8_M_TILE = 64  # rows per gpbs_hip_fp8_linear launch


def quant_rows_fp8(x: torch.Tensor):
    """Per-row symmetric e4m3fn quantisation on device: returns (q [rows, K]
    float8_e4m3fn, scale [rows] fp32) with scale = absmax / 448."""
    x = x.contiguous()
    _need(x, "quant_rows_fp8 x")
    K = x.shape[-1]
    if K % 8:
        raise ValueError(f"quant_rows_fp8: K={K} must be a multiple of 8")
    rows = x.numel() // K
    q = torch.empty(x.shape, dtype=torch.float8_e4m3fn, device=x.device)
    s = torch.empty(x.shape[:-1], dtype=torch.float32, device=x.device)
    _check(lib().gpbs_hip_quant_rows_fp8(_ptr(x), _ptr(q), _ptr(s), rows, K, _stream()), "quant_rows_fp8")
    return q, s


def quant_rows_fp8_ref(x: torch.Tensor):
    """fp32 PyTorch reference of quant_rows_fp8 (runs on CPU too)."""
    xf = x.float()
    amax = xf.abs().amax(-1)
    s = torch.where(amax > 0, amax / FP8_MAX, torch.ones_like(amax))
    inv = torch.where(amax > 0, FP8_MAX / amax, torch.ones_like(amax))  # multiply, as the kernel does
    q = (xf * inv.unsqueeze(-1)).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    return q, s


class Fp8Weight:
    """A linear weight [N, K] stored as e4m3fn rows plus per-output-channel scales."""

    def __init__(self, w: torch.Tensor):
        w = w.detach().to(torch.bfloat16).contiguous()
        self.N, self.K = w.shape
        if self.N % 16 or self.K % 256:
            raise ValueError(f"Fp8Weight: [N={self.N}, K={self.K}] needs N % 16 == 0 and K % 256 == 0")
        q, self.s = quant_rows_fp8(w) if w.is_cuda else quant_rows_fp8_ref(w)
        self.qs = self.shuffle(q)  # the only stored copy: the kernel's lane-order layout

    # Kernel layout: [N/16 strips][K/256 blocks][4 steps u][4 lane groups g][16 rows r][16 B];
    # lane l = 16 g + r of the wave that owns (strip, block) reads the 16 bytes
    # W[16 strip + r][256 block + 64 u + 16 g : +16] at step u, so each load
    # instruction is one contiguous 1 KiB run.
    def shuffle(self, q: torch.Tensor) -> torch.Tensor:
        b = q.view(torch.uint8).view(self.N // 16, 16, self.K // 256, 4, 4, 16)
        return b.permute(0, 2, 3, 4, 1, 5).contiguous().view(torch.float8_e4m3fn).view(self.N, self.K)

    @property
    def q(self) -> torch.Tensor:
        """Row-major [N, K] e4m3fn view (a copy; for references and tests)."""
        b = self.qs.view(torch.uint8).view(self.N // 16, self.K // 256, 4, 4, 16, 16)
        return b.permute(0, 4, 1, 2, 3, 5).contiguous().view(torch.float8_e4m3fn).view(self.N, self.K)

    def nbytes(self) -> int:
        return self.qs.numel() + 4 * self.s.numel()


def fp8_linear_q(xq: torch.Tensor, sx: torch.Tensor, w: Fp8Weight, resid: Optional[torch.Tensor] = None
                 ) -> torch.Tensor:
    """y = (xq @ Wq^T) * sx[m] * sw[n] (+ resid, fused into the epilogue) on
    already-quantised rows (the output of quant_rows_fp8 / rmsnorm_quant_fp8 /
    swiglu_quant_fp8); bf16 out."""
    lead = xq.shape[:-1]
    if xq.dtype != torch.float8_e4m3fn or xq.shape[-1] != w.K or not xq.is_contiguous():
        raise ValueError(f"fp8_linear_q: need contiguous e4m3fn [..., {w.K}], got {xq.dtype} {tuple(xq.shape)}")
    M = xq.numel() // w.K
    y = torch.empty(*lead, w.N, dtype=torch.bfloat16, device=xq.device)
    L, st = lib(), _stream()
    if resid is not None:
        _need(resid, "fp8_linear_q resid")
        if resid.numel() != M * w.N or M > FP8_M_TILE:
            raise ValueError(f"fp8_linear_q: resid {tuple(resid.shape)} for [{M}, {w.N}] (M <= {FP8_M_TILE})")
        _check(L.gpbs_hip_fp8_linear_res(_ptr(xq), _ptr(sx), _ptr(w.qs), _ptr(w.s), _ptr(y), _ptr(resid), M, w.N,
                                         w.K, st), "fp8_linear_res")
        return y
    if M <= FP8_M_TILE:
        _check(L.gpbs_hip_fp8_linear(_ptr(xq), _ptr(sx), _ptr(w.qs), _ptr(w.s), _ptr(y), M, w.N, w.K, st),
               "fp8_linear")
        return y
    x2, s2, y2 = xq.view(M, w.K), sx.reshape(M), y.view(M, w.N)
    for m0 in range(0, M, FP8_M_TILE):
        m1 = min(M, m0 + FP8_M_TILE)
        _check(L.gpbs_hip_fp8_linear(_ptr(x2[m0:m1]), _ptr(s2[m0:m1]), _ptr(w.qs), _ptr(w.s), _ptr(y2[m0:m1]),
                                     m1 - m0, w.N, w.K, st), "fp8_linear")
    return y


def fp8_linear(x: torch.Tensor, w: Fp8Weight) -> torch.Tensor:
    """y = x @ W^T with W in fp8 and x quantised per token to fp8 on the fly;
    fp32 MFMA accumulation, bf16 output.  x [..., K] bf16."""
    xq, sx = quant_rows_fp8(x)
    return fp8_linear_q(xq, sx, w)


def rmsnorm_quant_fp8(x: torch.Tensor, w: torch.Tensor, eps: float):
    """e4m3 rows of rmsnorm(x) * w plus their scales, in one kernel."""
    x = x.contiguous()
    _need(x, "rmsnorm_quant_fp8 x")
    dim = x.shape[-1]
    w = w.to(torch.bfloat16).contiguous()
    if w.numel() != dim or dim % 8:
        raise ValueError(f"rmsnorm_quant_fp8: weight {tuple(w.shape)} vs dim {dim}")
    q = torch.empty(x.shape, dtype=torch.float8_e4m3fn, device=x.device)
    s = torch.empty(x.shape[:-1], dtype=torch.float32, device=x.device)
    _check(lib().gpbs_hip_rmsnorm_quant_fp8(_ptr(x), _ptr(w), _ptr(q), _ptr(s), x.numel() // dim, dim,
                                            C.c_float(eps), _stream()), "rmsnorm_quant_fp8")
    return q, s


def swiglu_quant_fp8(gu: torch.Tensor):
    """e4m3 rows of silu(gu[..., :F]) * gu[..., F:] plus their scales (gu is the
    packed gate|up linear output, read in place)."""
    gu = gu.contiguous()
    _need(gu, "swiglu_quant_fp8 gu")
    F2 = gu.shape[-1]
    if F2 % 16:
        raise ValueError(f"swiglu_quant_fp8: packed width {F2} must be a multiple of 16")
    q = torch.empty(*gu.shape[:-1], F2 // 2, dtype=torch.float8_e4m3fn, device=gu.device)
    s = torch.empty(gu.shape[:-1], dtype=torch.float32, device=gu.device)
    _check(lib().gpbs_hip_swiglu_quant_fp8(_ptr(gu), _ptr(q), _ptr(s), gu.numel() // F2, F2 // 2, _stream()),
           "swiglu_quant_fp8")
    return q, s


def fp8_linear_ref(x: torch.Tensor, w: Fp8Weight) -> torch.Tensor:
    """fp32 reference of fp8_linear on the same quantised operands."""
    xq, sx = quant_rows_fp8_ref(x.reshape(-1, w.K))
    acc = xq.float() @ w.q.float().t()
    return (acc * sx.unsqueeze(1) * w.s.float().unsqueeze(0)).view(*x.shape[:-1], w.N)
