"""Torch-facing wrappers of the Llama tenant kernels (csrc/hip/llm_kernels.hip).

Inference-only (no autograd): the decode path of ``LlamaDecoder``.  The
library must load on a GPU box -- shape/dtype violations raise instead of
falling back to eager PyTorch.
"""
from __future__ import annotations

import ctypes as C

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
