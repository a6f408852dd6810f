"""Torch-facing wrappers of the gfx950 HIP kernels in libgpbs_hip.so.

These are the native hot ops of gpbs: the partition-aware MFMA GEMM and
streaming kernels that tenants run, and the scheduler's counter-reduce /
adapt / partition-switch kernels.  On a GPU box the library MUST load: the
ops raise instead of falling back to eager PyTorch.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from .. import _native as N

GATE_NONE, GATE_TABLE = 0, 1
WQ_BYTES = 64


def lib():
    L = N.load_hip(required=True)
    if L is None:
        raise RuntimeError("libgpbs_hip.so is not available (build with `python -m pbs_amd.build`)")
    return L


def _ptr(t: Optional[torch.Tensor]):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc})")


def work_queue(device=None) -> torch.Tensor:
    return torch.zeros(WQ_BYTES // 4, dtype=torch.int32, device=device or "cuda")


def status_word() -> torch.Tensor:
    return torch.zeros(1, dtype=torch.int32).pin_memory()


def gemm_bf16(A: torch.Tensor, Bt: torch.Tensor, out: Optional[torch.Tensor] = None, *, table=None, tenant: int = 0,
              counters=None, grid: int = 0, stream=None) -> torch.Tensor:
    """C = A @ Bt.T  (A: [M,K] bf16, Bt: [N,K] bf16) on MFMA, fp32 accumulation."""
    assert A.dtype == torch.bfloat16 and Bt.dtype == torch.bfloat16 and A.is_cuda
    M, K = A.shape
    Nn, K2 = Bt.shape
    if K != K2 or M % 128 or Nn % 128 or K % 64:
        raise ValueError(f"gemm_bf16 needs M,N % 128 == 0 and K % 64 == 0, got {A.shape} x {Bt.shape}")
    A = A.contiguous()
    Bt = Bt.contiguous()
    if out is None:
        out = torch.empty(M, Nn, dtype=torch.bfloat16, device=A.device)
    q = work_queue(A.device)
    rc = lib().gpbs_hip_gemm_bf16(_ptr(A), _ptr(Bt), _ptr(out), M, Nn, K, _ptr(q), table,
                                  GATE_TABLE if table else GATE_NONE, tenant, counters, None, grid, _stream(stream))
    _check(rc, "gemm_bf16")
    return out


def stream_copy(src: torch.Tensor, dst: torch.Tensor, *, chunk_bytes: int = 1 << 19, table=None, tenant: int = 0,
                counters=None, grid: int = 0, stream=None, mode_extra: int = 0):
    """``mode_extra``: gate-mode bits OR-ed in when ``table`` is given
    (e.g. GATE_DEVTABLE | GATE_HOLD for a VRAM table with the hold word)."""
    nbytes = src.numel() * src.element_size()
    assert dst.numel() * dst.element_size() >= nbytes and nbytes % 16 == 0
    q = work_queue(src.device)
    rc = lib().gpbs_hip_stream_copy(_ptr(src), _ptr(dst), nbytes, chunk_bytes, _ptr(q), table,
                                    (GATE_TABLE | mode_extra) if table else GATE_NONE, tenant, counters, None, grid,
                                    _stream(stream))
    _check(rc, "stream_copy")
    return dst


def reduce_bf16(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None, *, chunk_bytes: int = 1 << 19,
                table=None, tenant: int = 0, counters=None, grid: int = 0, stream=None) -> torch.Tensor:
    assert a.dtype == torch.bfloat16 and a.shape == b.shape
    if out is None:
        out = torch.empty_like(a)
    nbytes = a.numel() * 2
    q = work_queue(a.device)
    rc = lib().gpbs_hip_reduce_bf16(_ptr(a), _ptr(b), _ptr(out), nbytes, chunk_bytes, _ptr(q), table,
                                    GATE_TABLE if table else GATE_NONE, tenant, counters, None, grid,
                                    _stream(stream))
    _check(rc, "reduce_bf16")
    return out


def gemv_bf16(W: torch.Tensor, x: torch.Tensor, out: Optional[torch.Tensor] = None, *, table=None, tenant: int = 0,
              counters=None, grid: int = 0, stream=None) -> torch.Tensor:
    R, K = W.shape
    assert x.shape == (K,) and W.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
    if out is None:
        out = torch.empty(R, dtype=torch.float32, device=W.device)
    q = work_queue(W.device)
    rc = lib().gpbs_hip_gemv_bf16(_ptr(W), _ptr(x), _ptr(out), R, K, _ptr(q), table,
                                  GATE_TABLE if table else GATE_NONE, tenant, counters, None, grid, _stream(stream))
    _check(rc, "gemv_bf16")
    return out


GATE_SPATIAL = 8
GATE_DEVTABLE, GATE_HOLD = 4, 64


def census(blocks: int = 2048, table=None, tenant: int = 0, stream=None, spatial: bool = False) -> torch.Tensor:
    """Per-workgroup (XCC_ID, HW_ID, owned, magic).  ``stream`` may be a torch
    stream or a raw hipStream_t handle (int / c_void_p, e.g. a CU-masked one)."""
    out = torch.zeros(blocks * 4, dtype=torch.int32, device="cuda")
    mode = (GATE_TABLE if table else GATE_NONE) | (GATE_SPATIAL if spatial and table else 0)
    s = C.c_void_p(stream if isinstance(stream, int) else stream.value) if isinstance(stream, (int, C.c_void_p)) \
        else _stream(stream)
    rc = lib().gpbs_hip_census(_ptr(out), blocks, table, mode, tenant, s)
    _check(rc, "census")
    return out.view(blocks, 4)


def half_cu_mask(h: int):
    """CU-mask words selecting CU half ``h`` (shader engines 2h, 2h+1) of every
    XCD: bit b = logical CU b/8 of XCD b%8, logical CU i on SE i%4."""
    words = [0] * 8
    for b in range(256):
        if ((b // 8) % 4) >> 1 == h:
            words[b // 32] |= 1 << (b % 32)
    return words


def cumask_stream(words, device: int = 0) -> int:
    arr = (C.c_uint32 * len(words))(*words)
    h = lib().gpbs_gpu_cumask_stream(device, arr, len(words), 0)
    if not h:
        raise RuntimeError("hipExtStreamCreateWithCUMask failed")
    return h


def counter_reduce(cnt: torch.Tensor, prev: torch.Tensor, ids: torch.Tensor, stream=None) -> torch.Tensor:
    """Device per-tenant counter deltas: cnt/prev int64 [64, 8, 4]; ids int32."""
    n = ids.numel()
    out = torch.zeros(n, 4, dtype=torch.int64, device=cnt.device)
    rc = lib().gpbs_hip_counter_reduce(_ptr(cnt), _ptr(prev), _ptr(ids), n, _ptr(out), _stream(stream))
    _check(rc, "counter_reduce")
    return out


def adapt_batch(states: torch.Tensor, deltas: torch.Tensor, spin_sum: torch.Tensor, spin_cnt: torch.Tensor,
                params: N.AdaptParams, stream=None) -> torch.Tensor:
    """Batched PBS adaptation on device.  states: uint8 [n, sizeof(AdaptState)]
    (device), updated in place; returns per-tenant encoded directions."""
    n = deltas.shape[0]
    dirs = torch.zeros(n, dtype=torch.int32, device=states.device)
    rc = lib().gpbs_hip_adapt(_ptr(states), _ptr(deltas), _ptr(spin_sum), _ptr(spin_cnt), n, C.byref(params),
                              _ptr(dirs), _stream(stream))
    _check(rc, "adapt")
    return dirs


def partition_switch(table_dev: torch.Tensor, epoch: int, owners, stream=None):
    arr = (C.c_uint * 8)(*[(o if o >= 0 else 0xFFFFFFFF) for o in owners])
    rc = lib().gpbs_hip_partition_switch(_ptr(table_dev), epoch, arr, _stream(stream))
    _check(rc, "partition_switch")
