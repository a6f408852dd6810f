"""ctypes bindings to the native libraries (libgpbs.so, libgpbs_hip.so).

The C ABI is declared in csrc/include/gpbs/gpbs.h; struct layouts here mirror
it field for field.  Libraries are loaded from the in-tree ``pbs_amd/lib``
(built by ``pbs_amd.build``) so GPU runs always load the in-tree ``.so``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

LIBDIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")

u32, i32, u64, i64 = C.c_uint32, C.c_int32, C.c_uint64, C.c_int64


class AdaptParams(C.Structure):
    _fields_ = [(n, u32) for n in ("threshold", "band_lo", "band_hi", "min_us", "max_us", "inc_us", "dec_us",
                                   "switch_boundary", "ticks_per_tslice", "spin_floor", "scale", "strict_ref",
                                   "grow_pct")]


class AtcParams(C.Structure):
    _fields_ = [(n, u32) for n in ("default_us", "min_us", "max_us", "zero_step_us", "climb_step_us",
                                   "climb_floor_us", "base_us", "slope_us", "alpha", "warmup", "apply_period_us",
                                   "wait_unit_ns")]


ABI_VERSION = 6  # GPBS_ABI_VERSION in csrc/include/gpbs/gpbs.h


class BootParams(C.Structure):
    _fields_ = [("sched", C.c_char * 16)] + [(n, i32) for n in (
        "tslice_us", "ratelimit_us", "smt_power_savings", "tickle_one_idle", "default_yield", "migration_delay_us",
        "metric_period_us", "slice_apply_us", "sim_clock", "pmu_refresh_us", "dom0_quirk", "heartbeat_timeout_us",
        "trace_capacity", "quantum_align_us", "coschedule", "class_period_us", "boost_exclusive",
        "class_split", "idle_skip", "class_dwell", "class_budget", "present_us", "sibling_steal", "class_steal", "class_fall",
        "shared_q_us", "class_pin_us", "region_q", "switch_floor_x", "switch_floor_max_us", "region_vt",
        "slo_cap", "probe_max_us", "mem_split")] + [("adapt", AdaptParams),
                                                                                    ("atc", AtcParams)]


class SchedExt(C.Structure):
    _fields_ = [(n, i32) for n in ("weight", "period_us", "slice_us", "latency_us", "extratime", "credit")]


class FilterEntry(C.Structure):
    _fields_ = [("spin", u64), ("inst", u64), ("miss", u64)]


class AdaptState(C.Structure):
    _fields_ = [("tslice_us", u32), ("tick_period_us", u32), ("window_left", u32), ("stable_count", u32),
                ("phase", u32), ("last_err", i32), ("last_curr", i64), ("last_win", i64),
                ("filter", FilterEntry * 5)]


COUNTER_SLOT_REFRESH = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(u64))
COUNTER_TENANT_DELTAS = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(u64))
COUNTER_ADAPT_BATCH = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(u64), C.POINTER(u64),
                                  C.POINTER(u64), C.POINTER(AdaptState), C.POINTER(AdaptParams))
COUNTER_ADAPT_LAUNCH = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(u64), C.POINTER(u64),
                                   C.POINTER(u64), C.POINTER(AdaptState), C.POINTER(AdaptParams))
COUNTER_ADAPT_HARVEST = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(AdaptState))


class ArincEntry(C.Structure):
    _fields_ = [("tenant", i32), ("slot", i32), ("runtime_ns", C.c_int64)]


class ArincSchedule(C.Structure):
    _fields_ = [("major_frame_ns", C.c_int64), ("num_entries", i32), ("is_explicit", i32),
                ("entries", ArincEntry * 64)]


class CounterOps(C.Structure):
    _fields_ = [("user", C.c_void_p), ("slot_refresh", COUNTER_SLOT_REFRESH),
                ("tenant_deltas", COUNTER_TENANT_DELTAS), ("adapt_batch", COUNTER_ADAPT_BATCH),
                ("adapt_launch", COUNTER_ADAPT_LAUNCH), ("adapt_harvest", COUNTER_ADAPT_HARVEST)]


ACT_ON_SWITCH = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, i32, i64)
ACT_ON_FLUSH = C.CFUNCTYPE(None, C.c_void_p, i64)
ACT_ON_PARK = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_int, C.c_int)


class ActuatorOps(C.Structure):
    _fields_ = [("user", C.c_void_p), ("on_switch", ACT_ON_SWITCH), ("on_flush", ACT_ON_FLUSH),
                ("on_park", ACT_ON_PARK)]


class TraceRecord(C.Structure):
    _fields_ = [("t_ns", u64), ("event", u32), ("cpu", u32), ("a", u32 * 4)]


class TenantInfo(C.Structure):
    _fields_ = [(n, i32) for n in ("id", "pool", "nslots", "weight", "cap", "paused", "alive", "active_slots")] + \
               [(n, u32) for n in ("tslice_us", "tick_period_us", "phase", "window_left")] + \
               [("last_err", i32), ("shutdown", i32), ("last_curr", i64), ("last_win", i64), ("pmc", u64 * 4),
                ("cache_miss_rate", u64), ("cpi", u64), ("spin_latency", u64), ("report_count", u64),
                ("pending_requests", u64), ("sched_count", u64), ("run_ns", i64), ("name", C.c_char * 64),
                ("online_slots", i32), ("budget_ctx", u32), ("budget_shared", i32), ("target_tslice_us", u32),
                ("switch_cost_us", u32), ("slo_us", u32), ("last_dispatch_us", u32)]


class SlotInfo(C.Structure):
    _fields_ = [(n, i32) for n in ("id", "tenant", "index", "processor", "pri", "flags", "runstate",
                                   "is_running", "credit", "on_runq")] + \
               [("pmc", u64 * 4), ("sched_count", u64), ("run_ns", i64), ("runnable_ns", i64),
                ("blocked_ns", i64), ("affinity", u64 * 4), ("class_home", i32), ("pause_flags", u32)]


class PartitionInfo(C.Structure):
    _fields_ = [(n, i32) for n in ("id", "gpu", "xcd", "pool", "curr_tenant", "curr_slot", "runq_len", "idle",
                                   "ctx", "reserved")] + \
               [("switches", u64)]


class LockProf(C.Structure):
    _fields_ = [(n, u64) for n in ("lock_cnt", "block_cnt", "time_block_ns", "time_hold_ns", "max_block_ns",
                                   "max_hold_ns", "handoffs")]


_lock = threading.Lock()
_core = None
class GangCfg(C.Structure):
    _fields_ = [("rank", C.c_int32), ("ntenants", C.c_int32), ("nmetric", C.c_int32), ("metric_every", C.c_int32),
                ("tenants", C.c_int32 * 32), ("metric_tenants", C.c_int32 * 32),
                ("epoch_ns", C.c_int64), ("slack_ns", C.c_int64), ("deadline_ns", C.c_int64),
                ("start_ns", C.c_int64), ("join_ns", C.c_int64), ("share", C.c_double), ("atc_pool", C.c_int32),
                ("wait_driven", C.c_int32), ("wait_on_frac", C.c_double), ("wait_hold_epochs", C.c_int32),
                ("reform", C.c_int32), ("roctx_push", C.c_void_p), ("roctx_pop", C.c_void_p)]


class GangStats(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("epochs", "sync_p50_ns", "sync_p99_ns", "sync_max_ns", "skew_p50_ns",
                                         "skew_max_ns", "timeouts", "degraded", "reforms", "members",
                                         "atc_global_us", "metric_syncs", "gang_switches", "error", "finished")]


_hip = None


def _proto(lib, name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


def core_path():
    """GPBS_CORE_LIB selects another build of the core (e.g. the ASan/TSan
    builds of ``python -m pbs_amd.build --sanitize=address``)."""
    return os.environ.get("GPBS_CORE_LIB") or os.path.join(LIBDIR, "libgpbs.so")


def hip_path():
    return os.path.join(LIBDIR, "libgpbs_hip.so")


def load_core(build_if_missing=True):
    """Load libgpbs.so (builds it in-tree on first use if absent)."""
    global _core
    with _lock:
        if _core is not None:
            return _core
        p = core_path()
        if build_if_missing and not os.environ.get("GPBS_CORE_LIB"):
            from . import build
            build.build_core()
        lib = C.CDLL(p, mode=C.RTLD_GLOBAL)
        E = C.c_void_p
        P = _proto
        P(lib, "gpbs_boot_defaults", None, C.POINTER(BootParams))
        P(lib, "gpbs_engine_create", E, C.POINTER(BootParams))
        P(lib, "gpbs_engine_destroy", None, E)
        P(lib, "gpbs_abi_version", C.c_int)
        if lib.gpbs_abi_version() != ABI_VERSION:  # struct layouts below would be wrong
            raise RuntimeError(f"{p}: ABI {lib.gpbs_abi_version()} != {ABI_VERSION}; rebuild (python -m pbs_amd.build)")
        P(lib, "gpbs_strerror", C.c_char_p, C.c_int)
        P(lib, "gpbs_partition_add", C.c_int, E, C.c_int, C.c_int)
        P(lib, "gpbs_partition_add_ctx", C.c_int, E, C.c_int, C.c_int, C.c_int)
        P(lib, "gpbs_num_partitions", C.c_int, E)
        P(lib, "gpbs_pool_create", C.c_int, E, C.c_char_p, C.c_char_p)
        P(lib, "gpbs_pool_destroy", C.c_int, E, C.c_int)
        P(lib, "gpbs_pool_rename", C.c_int, E, C.c_int, C.c_char_p)
        P(lib, "gpbs_pool_find", C.c_int, E, C.c_char_p)
        P(lib, "gpbs_pool_assign", C.c_int, E, C.c_int, C.c_int)
        P(lib, "gpbs_pool_unassign", C.c_int, E, C.c_int, C.c_int)
        P(lib, "gpbs_pool_info", C.c_int, E, C.c_int, C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.POINTER(u64),
          C.POINTER(C.c_int))
        P(lib, "gpbs_pool_list", C.c_int, E, C.POINTER(C.c_int), C.c_int)
        P(lib, "gpbs_partition_info", C.c_int, E, C.c_int, C.POINTER(PartitionInfo))
        P(lib, "gpbs_tenant_create", C.c_int, E, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int)
        P(lib, "gpbs_tenant_destroy", C.c_int, E, C.c_int)
        P(lib, "gpbs_tenant_find", C.c_int, E, C.c_char_p)
        P(lib, "gpbs_tenant_list", C.c_int, E, C.POINTER(C.c_int), C.c_int)
        P(lib, "gpbs_tenant_move", C.c_int, E, C.c_int, C.c_int)
        P(lib, "gpbs_tenant_pause", C.c_int, E, C.c_int)
        P(lib, "gpbs_tenant_unpause", C.c_int, E, C.c_int)
        P(lib, "gpbs_tenant_set_nslots", C.c_int, E, C.c_int, C.c_int)
        P(lib, "gpbs_slot_id", C.c_int, E, C.c_int, C.c_int)
        P(lib, "gpbs_slot_wake", C.c_int, E, C.c_int, C.c_int)
        P(lib, "gpbs_slot_block", C.c_int, E, C.c_int, C.c_int)
        P(lib, "gpbs_slot_yield", C.c_int, E, C.c_int, C.c_int)
        P(lib, "gpbs_slot_pin", C.c_int, E, C.c_int, C.c_int, C.POINTER(u64))
        P(lib, "gpbs_tenant_info", C.c_int, E, C.c_int, C.POINTER(TenantInfo))
        P(lib, "gpbs_slot_info", C.c_int, E, C.c_int, C.POINTER(SlotInfo))
        P(lib, "gpbs_tenant_adapt_state", C.c_int, E, C.c_int, C.POINTER(AdaptState), C.c_int)
        P(lib, "gpbs_tenant_heartbeat", C.c_int, E, C.c_int)
        P(lib, "gpbs_sched_credit_get", C.c_int, E, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int))
        P(lib, "gpbs_sched_credit_set", C.c_int, E, C.c_int, C.c_int, C.c_int)
        P(lib, "gpbs_sched_ext", C.c_int, E, C.c_int, C.c_int, C.POINTER(SchedExt))
        P(lib, "gpbs_atc_sync", C.c_int, E, C.c_int, C.c_int)
        P(lib, "gpbs_arinc653_set", C.c_int, E, C.c_int, C.POINTER(ArincSchedule))
        P(lib, "gpbs_arinc653_get", C.c_int, E, C.c_int, C.POINTER(ArincSchedule))
        P(lib, "gpbs_sched_params_get", C.c_int, E, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int))
        P(lib, "gpbs_sched_params_set", C.c_int, E, C.c_int, C.c_int, C.c_int)
        P(lib, "gpbs_sched_name", C.c_int, E, C.c_int, C.c_char_p, C.c_int)
        P(lib, "gpbs_report_wait", C.c_int, E, C.c_int, u64, C.c_int)
        P(lib, "gpbs_report_requests", C.c_int, E, C.c_int, u64)
        P(lib, "gpbs_set_counter_ops", C.c_int, E, C.POINTER(CounterOps))
        P(lib, "gpbs_set_actuator_ops", C.c_int, E, C.POINTER(ActuatorOps))
        P(lib, "gpbs_backend_mux_add", C.c_int, E, C.c_int, C.c_int, C.POINTER(ActuatorOps), C.POINTER(CounterOps))
        P(lib, "gpbs_backend_mux_clear", C.c_int, E)
        P(lib, "gpbs_backend_mux_count", C.c_int, E)
        P(lib, "gpbs_fault_fire", i64, E, C.c_char_p)
        P(lib, "gpbs_gang_timeout", C.c_int, E, u32, u32, u32)
        P(lib, "gpbs_gang_shm_open", C.c_void_p, C.c_char_p, C.c_int, C.c_int, C.c_int)
        P(lib, "gpbs_gang_shm_allgather", C.c_int, C.c_void_p, u64, C.POINTER(i64), C.POINTER(i64), i64)
        P(lib, "gpbs_gang_shm_close", None, C.c_void_p)
        P(lib, "gpbs_gang_shm_reform", C.c_int, C.c_void_p, i64, i64, C.POINTER(u64), C.POINTER(u64))
        P(lib, "gpbs_gang_coord_start", C.c_void_p, E, C.c_void_p, C.c_int, C.c_int, C.POINTER(GangCfg))
        P(lib, "gpbs_gang_coord_stop", C.c_int, C.c_void_p, i64)
        P(lib, "gpbs_gang_coord_running", C.c_int, C.c_void_p)
        P(lib, "gpbs_gang_coord_stats", C.c_int, C.c_void_p, C.POINTER(GangStats))
        P(lib, "gpbs_gang_coord_tenant", C.c_int, C.c_void_p, C.c_int, C.POINTER(i64))
        P(lib, "gpbs_gang_coord_metrics", C.c_int, C.c_void_p, C.c_int, C.POINTER(i64), C.POINTER(i64))
        P(lib, "gpbs_gang_coord_history", C.c_int, C.c_void_p, C.POINTER(i64), C.POINTER(C.c_int32), C.c_int)
        P(lib, "gpbs_gang_coord_destroy", None, C.c_void_p)
        P(lib, "gpbs_slot_set_pmc", C.c_int, E, C.c_int, C.POINTER(u64))
        P(lib, "gpbs_now", i64, E)
        P(lib, "gpbs_advance", C.c_int, E, i64)
        P(lib, "gpbs_start", C.c_int, E)
        P(lib, "gpbs_stop", C.c_int, E)
        P(lib, "gpbs_poll", C.c_int, E)
        P(lib, "gpbs_next_event", i64, E)
        P(lib, "gpbs_debug_keys", C.c_int, E, C.c_char_p, C.c_char_p, C.c_int)
        P(lib, "gpbs_dmesg", C.c_int, E, C.c_char_p, C.c_int, C.c_int)
        P(lib, "gpbs_trace_read", C.c_int, E, C.POINTER(u64), C.POINTER(TraceRecord), C.c_int, C.POINTER(u64))
        P(lib, "gpbs_trace_set_mask", C.c_int, E, u64)
        P(lib, "gpbs_trace_emit", C.c_int, E, u32, u32, u32, u32, u32, u32)
        P(lib, "gpbs_perfc_count", C.c_int)
        P(lib, "gpbs_perfc_name", C.c_char_p, C.c_int)
        P(lib, "gpbs_perfc_read", C.c_int, E, C.POINTER(u64), C.c_int)
        P(lib, "gpbs_perfc_reset", C.c_int, E)
        P(lib, "gpbs_check_invariants", C.c_int, E, C.c_char_p, C.c_int)
        P(lib, "gpbs_lockprof", C.c_int, E, C.POINTER(LockProf), C.c_int)
        P(lib, "gpbs_watchdog", C.c_int, E, C.c_int, u32, u32)
        # host-side adaptation helpers (oracle parity tests)
        P(lib, "gpbs_adapt_init", None, C.POINTER(AdaptState), C.POINTER(AdaptParams), u32)
        P(lib, "gpbs_adapt_update", C.c_int, C.POINTER(AdaptState), C.POINTER(AdaptParams), u64, u64, u64, u64)
        # ipc: control pages, CPU counters/gates (optional components)
        for binder in (_bind_ipc, _bind_counters):
            try:
                binder(lib)
            except AttributeError:
                pass
        _core = lib
        return lib


def _bind_ipc(lib):
    P = _proto
    P(lib, "gpbs_ctl_create", C.c_void_p, C.c_char_p, C.c_int)
    P(lib, "gpbs_ctl_open", C.c_void_p, C.c_char_p)
    P(lib, "gpbs_ctl_close", None, C.c_void_p, C.c_int)
    P(lib, "gpbs_ctl_ntenants", C.c_int, C.c_void_p)
    P(lib, "gpbs_ctl_publish", None, C.c_void_p, C.c_int, u32, u64, u32, i32, i32, u32)
    P(lib, "gpbs_ctl_read", C.c_int, C.c_void_p, C.c_int, C.POINTER(u32), C.POINTER(u64), C.POINTER(u32),
      C.POINTER(i32), C.POINTER(i32), C.POINTER(u32))
    P(lib, "gpbs_gang_set", C.c_int, C.c_void_p, C.c_int, C.c_int, i64)
    P(lib, "gpbs_tenant_class", C.c_int, C.c_void_p, C.c_int)
    P(lib, "gpbs_tenant_bound_stats", C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_uint64), C.c_int)
    P(lib, "gpbs_tenant_measure", C.c_int, C.c_void_p, C.c_int, C.c_uint32)
    P(lib, "gpbs_tenant_switch_cost", C.c_int, C.c_void_p, C.c_int, C.c_uint64)
    P(lib, "gpbs_tenant_slo", C.c_int, C.c_void_p, C.c_int, C.c_uint32)
    P(lib, "gpbs_tenant_vpmu", C.c_int, C.c_void_p, C.c_int, C.POINTER(u64))
    P(lib, "gpbs_fault_set", C.c_int, C.c_void_p, C.c_char_p)
    P(lib, "gpbs_fault_hits", C.c_int, C.c_void_p, C.POINTER(u64), C.c_int)
    P(lib, "gpbs_ctl_report", C.c_int, C.c_void_p, C.c_int, u64, u32, u32)
    P(lib, "gpbs_ctl_read_mask", C.c_int, C.c_void_p, C.c_int, C.POINTER(u64), C.POINTER(u32))
    P(lib, "gpbs_ctl_read_vpmu", C.c_int, C.c_void_p, C.c_int, C.POINTER(u64), C.POINTER(u64), C.POINTER(u32),
      C.POINTER(i32), C.POINTER(u32), C.POINTER(u32))
    P(lib, "gpbs_ctl_drain", C.c_int, C.c_void_p, C.c_int, C.POINTER(u64), C.POINTER(u32), C.c_int)
    P(lib, "gpbs_ctl_heartbeat", None, C.c_void_p, C.c_int, u64, u32)
    P(lib, "gpbs_ctl_status", C.c_int, C.c_void_p, C.c_int, C.POINTER(u64), C.POINTER(u64), C.POINTER(u32),
      C.POINTER(u32))
    P(lib, "gpbs_ctl_set_counters", None, C.c_void_p, C.c_int, C.POINTER(u64))
    P(lib, "gpbs_ctl_get_counters", None, C.c_void_p, C.c_int, C.POINTER(u64))
    P(lib, "gpbs_ctl_wait_gate", C.c_int, C.c_void_p, C.c_int, i64)
    P(lib, "gpbs_ctl_ring", None, C.c_void_p, C.c_int)
    P(lib, "gpbs_ctl_doorbell_wait", C.c_int, C.c_void_p, C.c_int, i64)
    P(lib, "gpbs_ctl_set_work", None, C.c_void_p, C.c_int, C.c_int)
    P(lib, "gpbs_ctl_bind", C.c_int, C.c_void_p, C.c_void_p)
    P(lib, "gpbs_ctl_assign", C.c_int, C.c_void_p, C.c_int, C.c_int)


def _bind_counters(lib):
    P = _proto
    P(lib, "gpbs_perf_open", C.c_void_p, C.c_int, C.c_int)
    P(lib, "gpbs_perf_read", C.c_int, C.c_void_p, C.POINTER(u64))
    P(lib, "gpbs_perf_mode", C.c_int, C.c_void_p)
    P(lib, "gpbs_perf_close", None, C.c_void_p)
    P(lib, "gpbs_perf_available", C.c_int)
    P(lib, "gpbs_gate_create", C.c_void_p, C.c_char_p)
    P(lib, "gpbs_gate_add_pid", C.c_int, C.c_void_p, C.c_int, C.c_int)
    P(lib, "gpbs_gate_set", C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int)
    P(lib, "gpbs_gate_stats", C.c_int, C.c_void_p, C.POINTER(u64), C.POINTER(u64))
    P(lib, "gpbs_gate_destroy", None, C.c_void_p)
    P(lib, "gpbs_gate_mode", C.c_int, C.c_void_p)
    P(lib, "gpbs_cpu_backend_create", C.c_void_p, C.c_void_p, C.c_void_p)
    P(lib, "gpbs_cpu_backend_map", C.c_int, C.c_void_p, C.c_int, C.c_int)
    P(lib, "gpbs_cpu_backend_add", C.c_int, C.c_void_p, C.c_int, C.c_int)
    P(lib, "gpbs_cpu_backend_destroy", None, C.c_void_p)


def load_hip(required=False):
    """Load libgpbs_hip.so.  On a GPU box (``required=True``) a missing or
    unloadable library raises: GPU paths never silently fall back to eager
    PyTorch."""
    global _hip
    with _lock:
        if _hip is not None:
            return _hip
    load_core()
    with _lock:
        p = hip_path()
        if not os.path.exists(p):
            try:
                from . import build
                build.build_hip()
            except Exception:
                if required:
                    raise
                return None
        try:
            _hip = C.CDLL(p, mode=C.RTLD_GLOBAL)
        except OSError:
            if required:
                raise
            return None
        from .ops import hipabi
        hipabi.bind(_hip)
        return _hip


def check(rc, what=""):
    """Raise GpbsError for negative return codes."""
    if isinstance(rc, int) and rc < 0:
        lib = load_core()
        msg = lib.gpbs_strerror(rc).decode()
        from .core.errors import GpbsError
        raise GpbsError(rc, f"{what}: {msg}" if what else msg)
    return rc
