"""ctypes prototypes of libgpbs_hip.so (csrc/hip/*.hip, csrc/hip/runtime.cpp)."""
from __future__ import annotations

import ctypes as C

from .. import _native as N

u32, i32, u64, i64 = C.c_uint32, C.c_int32, C.c_uint64, C.c_int64
vp = C.c_void_p


class RunnerCfg(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("kind", "tenant", "gate", "priority", "depth", "grid", "M", "N", "K",
                                       "chunk_bytes", "engine_wake", "reserved")] + \
               [("bytes", C.c_ulonglong), ("a", vp), ("b", vp), ("c", vp)] + \
               [(n, C.c_int) for n in ("alt_kind", "alt_M", "alt_N", "alt_K", "alt_chunk_bytes", "alt_reserved")] + \
               [("alt_bytes", C.c_ulonglong), ("alt_a", vp), ("alt_b", vp), ("alt_c", vp)]


class RunnerStats(C.Structure):
    _fields_ = [(n, u64) for n in ("units_done", "launches", "relaunches", "waits_owner", "submitted")] + \
               [(n, i64) for n in ("busy_ns", "wait_owner_ns", "first_start_ns", "last_done_ns", "lat_sum_ns",
                                   "lat_max_ns")] + [("lat_count", u64), ("units_alt", u64)] + \
               [("drain_sum_ns", i64), ("drain_max_ns", i64), ("drain_count", u64)]


KIND = {"gemm": 1, "stream": 2, "reduce": 3, "gemv": 4, "allreduce": 5}


def _p(lib, name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)


def bind(lib):
    _p(lib, "gpbs_roctx_push", C.c_int, C.c_char_p)
    _p(lib, "gpbs_roctx_pop", C.c_int)
    _p(lib, "gpbs_roctx_mark", None, C.c_char_p)
    _p(lib, "gpbs_gpu_switch_latency", C.c_int, vp, C.c_int, C.c_int, vp)
    # raw kernels
    _p(lib, "gpbs_hip_gemm_bf16", C.c_int, vp, vp, vp, C.c_int, C.c_int, C.c_int, vp, vp, C.c_uint, C.c_uint, vp, vp,
       C.c_int, vp)
    _p(lib, "gpbs_hip_stream_copy", C.c_int, vp, vp, C.c_ulonglong, C.c_uint, vp, vp, C.c_uint, C.c_uint, vp, vp,
       C.c_int, vp)
    _p(lib, "gpbs_hip_reduce_bf16", C.c_int, vp, vp, vp, C.c_ulonglong, C.c_uint, vp, vp, C.c_uint, C.c_uint, vp, vp,
       C.c_int, vp)
    _p(lib, "gpbs_hip_gemv_bf16", C.c_int, vp, vp, vp, C.c_int, C.c_int, vp, vp, C.c_uint, C.c_uint, vp, vp, C.c_int,
       vp)
    _p(lib, "gpbs_hip_set_gemm_opts", C.c_int, C.c_int)
    _p(lib, "gpbs_hip_set_reduce_opts", C.c_int, C.c_int)
    _p(lib, "gpbs_hip_set_stream_opts", C.c_int, C.c_int)
    _p(lib, "gpbs_hwc_init", C.c_int, C.c_char_p)
    _p(lib, "gpbs_hwc_init_gpu", C.c_int, C.c_char_p, C.c_int)
    _p(lib, "gpbs_hwc_start", C.c_int)
    _p(lib, "gpbs_hwc_active", C.c_int)
    _p(lib, "gpbs_hwc_trace_enable", C.c_int, C.c_int)
    _p(lib, "gpbs_hwc_trace_stats", C.c_int, C.c_char_p, C.c_int, C.c_int)
    _p(lib, "gpbs_hwc_sample", C.c_int, C.POINTER(C.c_uint64), C.c_int)
    _p(lib, "gpbs_hwc_stop", C.c_int)
    _p(lib, "gpbs_gpu_set_hwc", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_gpu_hwc_stats", C.c_int, vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_double))
    _p(lib, "gpbs_hwc_sample_se", C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64))
    _p(lib, "gpbs_hwc_slot_per_se", C.c_int, C.c_int)
    _p(lib, "gpbs_hwc_agent", C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_int))
    _p(lib, "gpbs_gpu_hwc_period", C.c_int, vp, C.c_int, C.c_int, C.POINTER(C.c_uint64))
    _p(lib, "gpbs_gpu_hwc_quality", C.c_int, vp, C.POINTER(C.c_uint64), C.POINTER(C.c_double), C.POINTER(C.c_int))
    _p(lib, "gpbs_gpu_hwc_tenant", C.c_int, vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double))
    _p(lib, "gpbs_gpu_hwc_reset", C.c_int, vp)
    _p(lib, "gpbs_gpu_hwc_clean", C.c_int, vp, C.c_int, C.POINTER(C.c_double))
    _p(lib, "gpbs_gpu_hwc_tenant_metric", C.c_int, vp, C.c_int, C.POINTER(C.c_double))
    _p(lib, "gpbs_gpu_set_share", C.c_int, vp, C.c_int, C.POINTER(C.c_int64))
    _p(lib, "gpbs_gpu_hwc_poll", C.c_int, vp)
    _p(lib, "gpbs_gpu_set_se_mode", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_hip_rmsnorm_bf16", C.c_int, vp, vp, vp, C.c_int, C.c_int, C.c_float, vp)
    _p(lib, "gpbs_hip_swiglu_bf16", C.c_int, vp, vp, vp, C.c_ulonglong, vp)
    _p(lib, "gpbs_hip_quant_rows_fp8", C.c_int, vp, vp, vp, C.c_int, C.c_int, vp)
    _p(lib, "gpbs_hip_rmsnorm_quant_fp8", C.c_int, vp, vp, vp, vp, C.c_int, C.c_int, C.c_float, vp)
    _p(lib, "gpbs_hip_swiglu_quant_fp8", C.c_int, vp, vp, vp, C.c_int, C.c_int, vp)
    _p(lib, "gpbs_hip_fp8_set_opts", C.c_int, C.c_int)
    _p(lib, "gpbs_hip_fp8_linear_res", C.c_int, vp, vp, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, vp)
    _p(lib, "gpbs_hip_fp8_linear", C.c_int, vp, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, vp)
    _p(lib, "gpbs_hip_rope_bf16_dpos", C.c_int, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp)
    _p(lib, "gpbs_hip_qkv_rope_cache", C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int,
       C.c_int, vp)
    _p(lib, "gpbs_hip_decode_attn", C.c_int, vp, vp, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
       C.c_int, C.c_float, vp)
    _p(lib, "gpbs_hip_rope_bf16", C.c_int, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp)
    _p(lib, "gpbs_hip_census", C.c_int, vp, C.c_int, vp, C.c_uint, C.c_uint, vp)
    _p(lib, "gpbs_hip_partition_switch", C.c_int, vp, C.c_uint, C.POINTER(C.c_uint), vp)
    _p(lib, "gpbs_hip_counter_reduce", C.c_int, vp, vp, vp, C.c_int, vp, vp)
    _p(lib, "gpbs_hip_adapt", C.c_int, vp, vp, vp, vp, C.c_int, vp, vp, vp)
    # runtime
    _p(lib, "gpbs_gpu_ctx_create", vp, C.c_int, C.c_int, C.c_int, C.c_int)
    _p(lib, "gpbs_gpu_set_nctx", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_gpu_set_table_mode", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_gpu_table_mode", C.c_int, vp)
    _p(lib, "gpbs_gpu_set_hold", C.c_int, vp, C.c_int, C.POINTER(C.c_uint64))
    _p(lib, "gpbs_gpu_force_hold", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_gpu_set_spatial", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_gpu_set_waveprio", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_gpu_set_lat_half", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_gpu_hwc_attr_stats", C.c_int, vp, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64))
    _p(lib, "gpbs_gpu_set_hwc_device", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_gpu_hwc_duty", C.c_int, vp, C.c_int, C.POINTER(u64))
    _p(lib, "gpbs_gpu_hwc_bursts", C.c_int, vp, C.POINTER(u64), C.POINTER(u64))
    _p(lib, "gpbs_gpu_hwc_budget_stats", C.c_int, vp, C.POINTER(u64))
    _p(lib, "gpbs_gpu_hwc_sampler", C.c_int, vp, C.c_int, C.c_int, C.c_int)
    _p(lib, "gpbs_gpu_param", C.c_int, vp, C.c_char_p, C.c_int)
    _p(lib, "gpbs_gpu_hwc_attr_timing", C.c_int, vp, C.POINTER(u64))
    _p(lib, "gpbs_gpu_hwc_measure_reqs", C.c_uint64, vp)
    _p(lib, "gpbs_gpu_hwc_align", C.c_int, vp, C.c_int, C.c_int, C.c_int, C.POINTER(u64))
    _p(lib, "gpbs_gpu_hwc_tenant_periods", C.c_int, vp, C.c_int, C.POINTER(u64), C.POINTER(C.c_double))
    _p(lib, "gpbs_gpu_switch_cost", C.c_int, vp, C.c_int, C.POINTER(i64))
    _p(lib, "gpbs_gpu_hwc_tenant_cadence", C.c_int, vp, C.c_int, C.POINTER(i64))
    _p(lib, "gpbs_gpu_cadence_ring", C.c_int, vp, C.POINTER(i64), C.c_int)
    _p(lib, "gpbs_gpu_block_probe", C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(i64))
    _p(lib, "gpbs_runner_queue", C.c_int, vp)
    _p(lib, "gpbs_gpu_masked_pool", C.c_int, C.POINTER(C.c_uint64), C.c_int)
    _p(lib, "gpbs_hip_masked_pool_selftest", C.c_int)
    _p(lib, "gpbs_hip_hwc_fold_selftest", C.c_int)
    _p(lib, "gpbs_hip_hwc_drained_selftest", C.c_int, C.c_int, C.c_int)
    _p(lib, "gpbs_hip_hwc_cadence_selftest", C.c_int)
    _p(lib, "gpbs_hip_masked_pool_prealloc", C.c_int, C.c_int, C.POINTER(C.c_int), C.c_int)
    _p(lib, "gpbs_gpu_adapt_stats", C.c_int, vp, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64))
    _p(lib, "gpbs_hip_hwc_attr_selftest", C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double))
    _p(lib, "gpbs_hip_hwc_attr_host_check", C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double))
    _p(lib, "gpbs_hip_hwc_attr_bench", C.c_int, C.c_int, C.POINTER(C.c_double))
    _p(lib, "gpbs_hip_adapt_pools_selftest", C.c_int, C.c_int)
    _p(lib, "gpbs_gpu_ctx_destroy", None, vp)
    _p(lib, "gpbs_gpu_attach", C.c_int, vp, vp, C.c_int, C.c_int)
    _p(lib, "gpbs_gpu_backend_ops", C.c_int, vp, vp, C.POINTER(N.ActuatorOps), C.POINTER(N.CounterOps), C.c_int)
    _p(lib, "gpbs_gpu_table", vp, vp)
    _p(lib, "gpbs_gpu_counters", vp, vp)
    _p(lib, "gpbs_gpu_set_owners", C.c_int, vp, C.POINTER(C.c_int))
    _p(lib, "gpbs_gpu_get_owners", C.c_int, vp, C.POINTER(C.c_int))
    _p(lib, "gpbs_gpu_read_counters", C.c_int, vp, C.c_int, C.POINTER(u64), C.POINTER(u64))
    _p(lib, "gpbs_gpu_stats", C.c_int, vp, C.POINTER(u64))
    _p(lib, "gpbs_gpu_ownership", C.c_int, vp, C.c_int, C.POINTER(i64), C.c_int)
    _p(lib, "gpbs_gpu_cumask_stream", vp, C.c_int, C.POINTER(C.c_uint32), C.c_int, C.c_int)
    _p(lib, "gpbs_gpu_stream_destroy", C.c_int, vp)
    _p(lib, "gpbs_runner_create", vp, vp, C.POINTER(RunnerCfg))
    _p(lib, "gpbs_runner_submit", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_runner_wait", C.c_int, vp, i64)
    _p(lib, "gpbs_runner_stats", C.c_int, vp, C.POINTER(RunnerStats))
    _p(lib, "gpbs_runner_latencies", C.c_int, vp, C.POINTER(i64), C.c_int, C.c_int)
    _p(lib, "gpbs_runner_reset_stats", C.c_int, vp)
    _p(lib, "gpbs_runner_set_gate", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_runner_cancel", i64, vp)
    _p(lib, "gpbs_runner_set_engine_wake", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_runner_stream", vp, vp)
    _p(lib, "gpbs_runner_set_phase", C.c_int, vp, C.c_int)
    _p(lib, "gpbs_coll_create", vp, C.c_int, C.c_int, C.c_int, C.c_ulonglong)
    _p(lib, "gpbs_coll_export", C.c_int, vp, vp)
    _p(lib, "gpbs_coll_handle_bytes", C.c_int)
    _p(lib, "gpbs_coll_open", C.c_int, vp, C.c_int, vp)
    _p(lib, "gpbs_coll_finalize", C.c_int, vp)
    _p(lib, "gpbs_coll_buffer", vp, vp, C.c_int)
    _p(lib, "gpbs_coll_destroy", None, vp)
    _p(lib, "gpbs_gangx_create", vp, C.c_int, C.c_int, C.c_int, C.c_int)
    _p(lib, "gpbs_gangx_handle_bytes", C.c_int)
    _p(lib, "gpbs_gangx_export", C.c_int, vp, vp)
    _p(lib, "gpbs_gangx_open", C.c_int, vp, C.c_int, vp)
    _p(lib, "gpbs_gangx_finalize", C.c_int, vp)
    _p(lib, "gpbs_gangx_exchange", C.c_int, vp, C.c_uint, C.POINTER(C.c_longlong), C.c_int,
       C.POINTER(C.c_longlong), C.c_longlong)
    _p(lib, "gpbs_gangx_stats", C.c_int, vp, C.POINTER(u64))
    _p(lib, "gpbs_gangx_destroy", None, vp)
    _p(lib, "gpbs_coll_copy", C.c_int, vp, C.c_int, vp, C.c_ulonglong, C.c_int)
    _p(lib, "gpbs_runner_destroy", None, vp)
