"""Co-run benchmark: the BASELINE.json headline metric.

"co-run slowdown (%) vs solo + aggregate throughput, 4-tenant mix at
1/2/4/8 GPU" (SURVEY §6 protocol; config #3 per GPU, weak scaling).

Per GPU rank, four tenants share one MI355X:

* ``gemm``  bf16 4096^3 MFMA GEMM (compute-bound)             native runner
* ``hbm``   1 GiB float4 copy (HBM-bound)                      native runner
* ``coll``  all-reduce tenant: RCCL all-reduce over xGMI when N > 1, the
            reduce-copy traffic kernel on one GPU              native runner / thread
* ``idle``  latency tenant: 8192^2 GEMV requests, 2 ms think time, closed loop

Protocol "steady" (default; SURVEY §6 weighted speedup): every throughput
tenant is kept backlogged for the whole run; a step is one ``step_ms``
window; over the K timed steps

  norm_perf_i = (units_i / t) / solo_rate_i    (idle tenant: solo/co-run p50 latency)
  slowdown_i  = 1 / norm_perf_i - 1            (per tenant, %)
  aggregate   = sum_i norm_perf_i over the throughput tenants

Protocol "quota" (round 1): a step gives each throughput tenant a quota that
takes ``target_ms`` solo and ends when all are done (t_i = its completion
time, norm_perf_i = T_i / t_i); early finishers idle, so late ones run the
step's tail alone, which rewards staggering completions rather than sharing.

``value`` = aggregate summed over all GPUs (whole-job, solo-equivalents).

Policies (same tenants, same box):
  none     default hardware sharing: every tenant launches ungated full-GPU grids
  static   equal static XCD split (2 XCDs per tenant, ARINC-653-like)
  gpbs     (flagship) counter-driven contention classes over shader-engine (SE)
           exclusive partitions, 4 per XCD, one owner each.  Live CDNA4
           counters, attributed by SE ownership in exclusive-ownership
           windows, drive the PBS phase detector and the contention class;
           the compute class owns SEs {0,1} of every XCD, each memory-class
           tenant one memory SE of every XCD (memory tenants never share an
           SE: per-SE load paths cap a stream at ~0.5 of HBM on one SE and
           ~0.93 on two, and time-sharing two SEs between memory tenants at
           ms quanta measured below splitting them); runners launch on
           CU-masked streams of their class half; the latency tenant runs
           outside the partitions, co-resident at raised wave priority
  credit-fixed   the same with a fixed credit quantum (PBS ablation: nothing
           is time-shared in this mix, so adaptive quanta change nothing)
  gpbs-ts  memory tenants alternate on the memory SEs {2,3} as one gang with
           PBS adaptive quanta (round-2 first flagship; credit-fixed-ts: same
           with a fixed quantum -- the PBS-quanta ablation)
  credit2  the SE partitions under credit2 (no classes)
  gpbs-boost  latency tenant inside the partitions (wake-BOOST revokes SEs)
  gpbs-ctx4   round-1 flagship: four co-resident issue contexts per XCD,
           parked gating, wave priority (counters attributed by time share)
  gpbs-ctx2 / gpbs-spatial / gpbs-x / gpbs-noprio / gpbs-nogang / gpbs1 /
  gpbs-exit / sedf   round-1 variants kept for ablations

Every timed run of a scheduler policy starts from a fresh engine (no
classes, credits or quanta carried over from an earlier run of the policy);
``fresh_engine=False`` keeps one engine per policy for the whole process.
"""
from __future__ import annotations

import json
import os
import statistics
import threading
import time
from dataclasses import dataclass
from typing import Callable, Dict, Optional

import torch

from ..core.config import MI355X_PROFILE
from ..core.engine import Engine
from ..runtime.gpu import XCDS, GpuContext, Runner

THROUGHPUT = ("gemm", "hbm", "coll")
TENANTS = (("gemm", 8), ("hbm", 8), ("coll", 8), ("idle", 8))  # one slot per XCD
# Tenant workloads (native runners; "coll" is the RCCL all-reduce tenant when
# N > 1).  "phase" alternates between a 4096^3 GEMM (compute-bound) and a
# 1 GiB stream copy (memory-bound) every phase_ms.
SPECS = {
    "gemm": dict(kind="gemm", M=4096, N=4096, K=4096),
    "gemm_b": dict(kind="gemm", M=4096, N=4096, K=4096),
    "gemm_s": dict(kind="gemm", M=2048, N=2048, K=2048),
    "hbm": dict(kind="stream", bytes=1 << 30),
    "hbm_b": dict(kind="stream", bytes=1 << 30),
    "hbm_s": dict(kind="stream", bytes=256 << 20),
    "mall": dict(kind="stream", bytes=96 << 20),
    "coll": dict(kind="reduce"),  # bytes = cfg.coll_bytes
    "phase": dict(kind="gemm", M=4096, N=4096, K=4096, alt=dict(kind="stream", bytes=1 << 30)),
    "idle": dict(kind="gemv"),
}
# Tenant mixes (BASELINE.json configs): "4mix" = config #3 (MFMA GEMM + HBM
# stream + all-reduce + latency-critical idle; the headline); "gemm2" =
# config #2; "phase" = a phase-changing mix (the "phase" tenant alternates
# compute <-> memory every phase_ms, the "hbm" tenant stops and starts every
# onoff_ms) -- what a counter-driven scheduler must follow and a hand-picked
# static layout cannot; "8mix" = config #4's 8-tenant mix on one GPU (3 GEMMs,
# 3 streams + the reduce/all-reduce, latency GEMV): more tenants per class
# than shader engines, so classes must time-share their SEs.
MIXES = {
    "4mix": {"tenants": TENANTS, "throughput": THROUGHPUT},
    "gemm2": {"tenants": (("gemm", 8), ("gemm_b", 8)), "throughput": ("gemm", "gemm_b")},
    "phase": {"tenants": (("gemm", 8), ("phase", 8), ("hbm", 8), ("idle", 8)),
              "throughput": ("gemm", "phase", "hbm"), "dynamic": True},
    # time-shared phase mix: the phase tenant flips into a
    # memory region that already holds two or three memory tenants (hbm on /
    # off), so the region is time-shared and PBS's re-arm moves quanta that
    # rotate real co-sharers
    "phase-ts": {"tenants": (("gemm", 8), ("phase", 8), ("hbm", 8), ("hbm_b", 8), ("coll", 8), ("idle", 8)),
                 "throughput": ("gemm", "phase", "hbm", "hbm_b", "coll"), "dynamic": True},
    "8mix": {"tenants": (("gemm", 8), ("gemm_b", 8), ("gemm_s", 8), ("hbm", 8), ("hbm_b", 8), ("hbm_s", 8),
                         ("coll", 8), ("idle", 8)),
             "throughput": ("gemm", "gemm_b", "gemm_s", "hbm", "hbm_b", "hbm_s", "coll")},
    # latency-SLO mix: the latency tenant is a co-sharer
    # of the time-shared memory region (gated on its partitions, woken per
    # request -- no latency lane), next to two HBM streamers and a tenant
    # whose working set (2 x 96 MiB) fits the 256 MiB MALL
    "slo": {"tenants": (("gemm", 8), ("hbm", 8), ("hbm_b", 8), ("mall", 8), ("idle", 8)),
            "throughput": ("gemm", "hbm", "hbm_b", "mall"), "slo_in_region": True,
            # p99 target of its 8192^2 GEMV requests (solo ~0.06 ms)
            "slo_p99_ms": 1.0},
}
# Alternative hand layouts (policy "static-se2"), probes of the layout space
STATIC_SE2 = {
    # slo: the launch-bound MALL-sized tenant on a memory SE of its own on
    # most XCDs, the two streams split the other memory SE
    "slo": {"gemm": (tuple(range(8)), (0, 1)), "hbm": ((0, 1, 2, 3), (2,)), "hbm_b": ((4, 5, 6, 7), (2,)),
            "mall": ((0, 1, 2, 3, 4, 5), (3,)), "idle": ((6, 7), (3,))},
}

# Hand-picked static shader-engine layouts (policy "static-se": no engine, no
# counters): tenant -> (XCDs, SEs) it owns.  The informed static alternative
# to the counter-driven layout: for the 4mix the compute tenant on SEs {0,1}
# and one memory SE per memory tenant (profiles/se_interfere_1gpu.jsonl
# g2|s1|r1, the best split measured).
_ALLX = tuple(range(8))
STATIC_SE = {
    "4mix": {"gemm": (_ALLX, (0, 1)), "hbm": (_ALLX, (2,)), "coll": (_ALLX, (3,))},
    "gemm2": {"gemm": (_ALLX, (0, 1)), "gemm_b": (_ALLX, (2, 3))},
    "phase": {"gemm": (_ALLX, (0, 1)), "phase": (_ALLX, (2,)), "hbm": (_ALLX, (3,))},
    "phase-ts": {"gemm": (_ALLX, (0, 1)), "phase": ((0, 1, 2, 3), (2,)), "hbm": ((4, 5, 6, 7), (2,)),
                 "hbm_b": ((0, 1, 2, 3), (3,)), "coll": ((4, 5, 6, 7), (3,))},
    "8mix": {"gemm": (_ALLX, (0,)), "gemm_b": (tuple(range(6)), (1,)), "gemm_s": ((6, 7), (1,)),
             "hbm": ((0, 1, 2, 3), (2,)), "hbm_b": ((4, 5, 6, 7), (2,)), "coll": ((0, 1, 2, 3), (3,)),
             "hbm_s": ((4, 5, 6, 7), (3,))},
    # the latency tenant gets dedicated memory SEs (idle between requests)
    "slo": {"gemm": (_ALLX, (0, 1)), "hbm": ((0, 1, 2, 3), (2,)), "hbm_b": ((4, 5, 6, 7), (2,)),
            "mall": ((0, 1, 2, 3), (3,)), "idle": ((4, 5, 6, 7), (3,))},
}


@dataclass
class CorunConfig:
    steps: int = 20
    warmup: int = 3
    target_ms: float = 30.0
    policies: tuple = ("none", "static", "gpbs")
    gemm_n: int = 4096
    hbm_bytes: int = 1 << 30
    coll_bytes: int = 256 << 20
    idle_rows: int = 8192
    idle_period_ms: float = 2.0
    depth: int = 2
    table_mode: str = "host"
    calib_units: int = 8
    gang_epoch_ms: float = 4.0   # N > 1: cross-GPU gang window length
    gang_share: float = 0.5      # fraction of epochs that are the all-reduce tenant's
    gang_transport: str = "shm"  # shm (one node, native) | dist (the "gang" process group: gloo or RCCL)
    gang_shm_base: str = ""      # region name prefix agreed by all ranks (a nonce broadcast by rank 0)
    gang_deadline_ms: float = 200.0
    gang_wait_driven: bool = False  # gang windows only while the coll tenant's K10 waits say its peers lag
    coll_impl: str = "ipc"       # N > 1 all-reduce tenant: "ipc" (gated gpbs kernel over IPC-mapped peer
                                 # buffers, csrc/hip/coll_kernels.hip) or "rccl" (torch.distributed, ungated)
    mix: str = "4mix"
    hw_counters: bool = False    # PBS metric from live hardware counters
    # "steady": every throughput tenant is kept backlogged for the whole timed
    # window (a step = one step_ms window); throughput_i = units done / time,
    # normalised by the solo rate -- the weighted speedup of SURVEY §6.
    # "quota" (round 1): a step gives each tenant a fixed quota and ends when
    # all are done, so early finishers idle and late ones run the tail alone.
    protocol: str = "steady"
    step_ms: float = 80.0
    fresh_engine: bool = True    # every run of a scheduler policy starts from a new engine
    phase_ms: float = 300.0      # mix "phase": the phase tenant alternates gemm <-> stream this often
    onoff_ms: float = 500.0      # mix "phase": the hbm tenant runs / stops for this long, alternately
    solo_steps: int = 0          # solo calibration windows (0: the co-run's K); warmup = the co-run's W
    mem_chunk: int = 0           # memory tenants' chunk bytes (0: the runner default, 512 KiB)
    kernel_trace: bool = False   # per-run in-process kernel trace (counters/hwc.py trace_stats)


# SE-exclusive flagship (the four partitions of an XCD are its shader engines,
# one owner each): the compute class owns SEs {0,1} of every XCD and the
# memory class SEs {2,3}, each class group gang-switched as a whole, memory
# tenants time-sharing their SEs under credit with PBS quanta, on
# counters attributed exactly by SE ownership
# (profiles/se_interfere_1gpu.jsonl, profiles/hwc/se_separation_probe.txt).
SE_OVERRIDES = {"class_split": 2, "idle_skip": 1}
# demand-driven SE budgets (csrc/core/engine.cpp budget_layout): the layout,
# not a slot count, sizes each tenant's share -- every tenant is created with
# one slot per partition and surplus slots go offline
BUDGET_OVERRIDES = {"class_split": 2, "idle_skip": 1, "class_budget": 2, "present_us": 10000}
SE_SLOTS = {"gemm": 16, "gemm_b": 16, "hbm": 16, "coll": 16, "idle": 8}
# "se8": memory tenants get 8 slots each -- one SE per XCD, so the credit
# scheduler places them on disjoint memory SEs instead of time-sharing both.
SE8_SLOTS = {"gemm": 16, "gemm_b": 16, "hbm": 8, "coll": 8, "idle": 8}

# Runtime path of the SE-budget policies (round 6): the
# partition table in fine-grained VRAM the host writes through the BAR (no
# k_partition_switch), the PBS update and the counter attribution on the host
# (the bit-exact twins of k_adapt / k_hwc_attribute), the modeled counter block
# read through the BAR -- the scheduler puts no kernel and no blit on the GPU's
# queues, so nothing it does waits behind the tenants' persistent grids
# (profiles/r6/s13_*: 0 scheduler dispatches vs ~1000 k_adapt/s at 35-60 us
# mean, 400+ us max, on the device path).  Every policy that lays out SE
# budgets runs the same path, so the ablations differ from the flagship in
# policy only.  RT_DEV: the round-5 device path (gpbs-dev).
RT = "bar,se,waveprio,latco,budget,latmem,hostsched"
RT_DEV = "device,se,waveprio,latco,budget,latmem"

POLICY_ENGINES = {
    # name: (issue contexts per XCD, engine overrides on top of MI355X_PROFILE,
    #        kernel gate mode, partition-table location + runtime options)
    # flagship: counter-driven SE budgets (csrc/core/engine.cpp budget_layout)
    # -- every present tenant gets shader engines sized from the classes
    # present; a class region with more tenants than its aligned blocks hold
    # is time-shared under credit with PBS adaptive quanta (class_budget 1);
    # runners launch on CU-masked class-half streams; the latency tenant runs
    # outside the partitions in the latency lane (its GEMV CU-masked to the
    # memory half, raised wave priority).  Uncrowded mixes (4mix, phase) lay
    # out exactly as gpbs-split; on the crowded 8mix time-sharing with PBS
    # quanta measured ahead of the XCD-block split on 3 of 4 boxes
    # (profiles/r3/8mix_queues_q8_*.json, bench_full_5rep_b.json, bench_all_pool_2rep.json).
    "gpbs": (4, dict(BUDGET_OVERRIDES, class_budget=1), True, RT),
    # crowded class regions split by whole-XCD blocks instead (class_budget 2)
    "gpbs-split": (4, dict(BUDGET_OVERRIDES), True, RT),
    # the flagship on round 5's device path (device table + k_partition_switch,
    # k_adapt, k_hwc_attribute), and with only the table moved to the BAR
    "gpbs-dev": (4, dict(BUDGET_OVERRIDES, class_budget=1), True, RT_DEV),
    # crowded memory regions split by partitions with a dedicated light
    # (latency) block (mem_split 1); gpbs-ms2 = the flagship's mem_split 2
    # (the light block overlaps the largest backlogged block)
    "gpbs-ms": (4, dict(BUDGET_OVERRIDES, class_budget=1, mem_split=1), True, RT),
    "gpbs-ms2": (4, dict(BUDGET_OVERRIDES, class_budget=1, mem_split=2), True, RT),
    "gpbs-bar": (4, dict(BUDGET_OVERRIDES, class_budget=1), True, "bar,se,waveprio,latco,budget,latmem"),
    # the flagship with a smaller hardware-sample budget (SAMPLER below)
    "gpbs-b1": (4, dict(BUDGET_OVERRIDES, class_budget=1), True, RT),
    "gpbs-b2": (4, dict(BUDGET_OVERRIDES, class_budget=1), True, RT),
    "credit-fixed": (4, dict(BUDGET_OVERRIDES, sched="credit-fixed"), True, RT),
    # round-3 name of the flagship on crowded mixes (time-shared, PBS quanta;
    # credit-fixed-ts: the fixed quantum)
    # the flagship with crowded memory regions time-shared (mem_split 0): the
    # layout ablation of round 6
    "gpbs-ts": (4, dict(BUDGET_OVERRIDES, class_budget=1, mem_split=0), True, RT),
    "credit-fixed-ts": (4, dict(BUDGET_OVERRIDES, class_budget=1, sched="credit-fixed"), True,
                        RT),
    # fixed per-class quanta (memory class max_us, compute class min_us), no
    # phase detector: what PBS's detector adds over a class -> quantum table
    "credit-classq": (4, dict(BUDGET_OVERRIDES, class_budget=1, sched="credit-classq"), True,
                      RT),
    # the ATC policy (X:xen/common/sched_credit_atc.c:291-543): one global
    # quantum for the pool, driven by the tenants' wait reports (K10); the
    # same time-shared budget layout as the flagship
    "atc": (4, dict(BUDGET_OVERRIDES, class_budget=1, sched="atc", region_vt=0), True,
            RT),
    "atc-vt": (4, dict(BUDGET_OVERRIDES, class_budget=1, sched="atc"), True, RT),
    "atc-nox": (4, dict(BUDGET_OVERRIDES, class_budget=1, sched="atc", class_steal=0), True,
                RT),
    # switch-cost probes: every quantum (fixed) or the adaptive floor at 4 ms
    "credit-fixed-ts4": (4, dict(BUDGET_OVERRIDES, class_budget=1, sched="credit-fixed", tslice_us=4000), True,
                         RT),
    "gpbs-f4": (4, dict(BUDGET_OVERRIDES, class_budget=1, adapt=dict(MI355X_PROFILE["adapt"], min_us=4000)), True,
                RT),
    # the class EWMA follows a drop at alpha 1/2 (boot class_fall=1)
    "gpbs-fall": (4, dict(BUDGET_OVERRIDES, class_budget=1, class_fall=1), True,
                  RT),
    # PBS quantum range stretched 3x at the top (memory tenants up to 33 ms)
    "gpbs-q33": (4, dict(BUDGET_OVERRIDES, class_budget=1,
                         adapt=dict(MI355X_PROFILE["adapt"], max_us=33000, inc_us=3000, dec_us=6000)), True,
                 RT),
    # long quanta everywhere: 30 ms fixed (the ATC default without its wait
    # feedback), and the PBS range moved up to 4-30 ms
    # (the equal-quantum ablations run credit ordering in the region,
    # region_vt 0: measured better for them than the flagship's region
    # virtual time -- 8mix fixed-30 1.388 vs 1.302, atc 1.388 vs 1.325,
    # profiles/r6/s2_8mix_vt_summary.txt)
    "credit-fixed-ts30": (4, dict(BUDGET_OVERRIDES, class_budget=1, sched="credit-fixed", tslice_us=30000,
                                  region_vt=0), True, RT),
    "gpbs-w": (4, dict(BUDGET_OVERRIDES, class_budget=1,
                       adapt=dict(MI355X_PROFILE["adapt"], min_us=4000, max_us=30000, inc_us=4000, dec_us=8000,
                                  switch_boundary=30000)), True, RT),
    # time-shared class regions rotate at >= 11 / 30 ms (boot shared_q_us)
    "gpbs-sq11": (4, dict(BUDGET_OVERRIDES, class_budget=1, region_q=1, shared_q_us=11000), True,
                  RT),
    # round 5's flagship: one region quantum (the co-sharers' largest adaptive
    # quantum, floored at a global 30 ms)
    "gpbs-sq30": (4, dict(BUDGET_OVERRIDES, class_budget=1, region_q=1, shared_q_us=30000, mem_split=0), True,
                  RT),
    # the long-quantum ablations with credit ordering the time-shared region
    # (region_vt 0: round 5's dispatch core)
    "gpbs-novt": (4, dict(BUDGET_OVERRIDES, class_budget=1, region_vt=0), True,
                  RT),
    # the PBS quantum without the measured switch-cost floors
    "gpbs-nofloor": (4, dict(BUDGET_OVERRIDES, class_budget=1, switch_floor_x=0), True,
                     RT),
    # credit-classq with the global 30 ms floor in time-shared regions (the
    # classq + floor ablation: what the class map does with round 5's floor)
    "credit-classq-f": (4, dict(BUDGET_OVERRIDES, class_budget=1, sched="credit-classq", shared_q_us=30000,
                                region_vt=0), True, RT),
    "credit-classq-fvt": (4, dict(BUDGET_OVERRIDES, class_budget=1, sched="credit-classq", shared_q_us=30000), True,
                          RT),
    "credit-fixed-ts30-vt": (4, dict(BUDGET_OVERRIDES, class_budget=1, sched="credit-fixed", tslice_us=30000), True,
                             RT),
    # PBS quantum range capped lower at the top (memory tenants up to 4 / 6 ms)
    "gpbs-max4": (4, dict(BUDGET_OVERRIDES, class_budget=1, adapt=dict(MI355X_PROFILE["adapt"], max_us=4000)), True,
                  RT),
    "gpbs-max6": (4, dict(BUDGET_OVERRIDES, class_budget=1, adapt=dict(MI355X_PROFILE["adapt"], max_us=6000)), True,
                  RT),
    # a tenant flapping between classes (3 changes within 2 s) is laid out in
    # the memory region until it settles (boot class_pin_us)
    "gpbs-pin": (4, dict(BUDGET_OVERRIDES, class_budget=1, class_pin_us=2000000), True,
                 RT),
    # class changes must persist 100 / 300 ms (class_dwell x class_period_us)
    # before a tenant is re-homed: flap damping for phase-changing tenants
    "gpbs-dwell50": (4, dict(BUDGET_OVERRIDES, class_budget=1, class_dwell=50), True,
                     RT),
    "gpbs-dwell150": (4, dict(BUDGET_OVERRIDES, class_budget=1, class_dwell=150), True,
                      RT),
    # the flagship under other counter-sampler policies (same engine and
    # layout; SAMPLER below): round-3 sampler (owner-change bursts, no budget,
    # no model fallback), and modeled counters only (no hardware sample)
    "gpbs-model": (4, dict(BUDGET_OVERRIDES, class_budget=1), True, RT),
    "gpbs-noalign": (4, dict(BUDGET_OVERRIDES, class_budget=1), True, RT),
    "gpbs-d5": (4, dict(BUDGET_OVERRIDES, class_budget=1), True, RT),
    # no cross-class steals by idle partitions (boot class_steal=0)
    "gpbs-nox": (4, dict(BUDGET_OVERRIDES, class_budget=1, class_steal=0), True,
                 RT),
    "gpbs-d10": (4, dict(BUDGET_OVERRIDES, class_budget=1), True, RT),
    # the same without the latency lane (GEMV co-resident on every CU)
    "gpbs-nolane": (4, dict(BUDGET_OVERRIDES), True, "device,se,waveprio,latco,budget"),
    # round-2 flagship: fixed class halves, memory tenants one SE each by
    # their bench-side slot count (se8)
    "gpbs-se8": (4, dict(SE_OVERRIDES), True, "device,se,waveprio,latco,se8"),
    "gpbs-share": (4, dict(SE_OVERRIDES), True, "device,se,waveprio,latco,se8,share"),
    # flagship + latency hold: the table in host-written VRAM (BAR), and the
    # memory-class tenants pause at their next unit boundary while a latency
    # request is in flight (the wake-BOOST analog for the GEMV tenant)
    # flagship + latency hold (memory-class tenants pause at their next unit
    # boundary while a latency request is in flight; BAR-written VRAM table)
    "gpbs-lat": (4, dict(BUDGET_OVERRIDES), True, "bar,se,waveprio,latco,budget,hold,latmem"),
    # round-2 time-shared variant: memory tenants alternate on SEs {2,3}
    "gpbs-ts-r2": (4, dict(SE_OVERRIDES), True, "device,se,waveprio,latco"),
    "credit-fixed-ts-r2": (4, dict(SE_OVERRIDES, sched="credit-fixed"), True, "device,se,waveprio,latco"),
    "credit2": (4, dict(SE_OVERRIDES, sched="credit2"), True, "device,se,waveprio,latco"),
    "gpbs-boost": (4, dict(SE_OVERRIDES), True, "device,se,waveprio"),
    "gpbs-host": (4, dict(SE_OVERRIDES), True, "host,se,waveprio,latco"),
    "gpbs-ctx4": (4, {}, "park", "device,waveprio"),
    "gpbs-x": (4, {"boost_exclusive": 1}, "park", "device,waveprio"),
    "gpbs-noprio": (4, {}, "park", "device"),
    "gpbs-ctx2": (2, {}, "park", "device"),
    "gpbs-spatial": (2, {}, "park", "device,spatial"),
    "gpbs-nogang": (4, dict(SE_OVERRIDES, coschedule=2), True, "device,se,waveprio"),
    "gpbs-exit": (2, {}, True, "host"),
    "gpbs1": (1, {"coschedule": 0}, True, "host"),
    "sedf": (4, dict(SE_OVERRIDES, sched="sedf"), True, "device,se,waveprio"),
}


# Counter-sampler policy per scheduler policy (GpuContext.set_hwc_sampler
# arguments; "model": no hardware samples, the modeled per-tile counters feed
# the metric).  Policies not listed run the process defaults (env / runtime).
SAMPLER = {
    # the round-4 sampler: no switch-aligned samples (periodic / phase bursts
    # only), the same calibrated fallback
    "gpbs-noalign": dict(align=0),
    "gpbs-model": "model",
    # background cadence: the duty cap (default 1 %) sets the period from the
    # ~0.2 ms sample cost; 5 % -> ~4 ms, 10 % -> ~2 ms (budget raised with it)
    "gpbs-d5": dict(budget_pct=8, duty=5),
    "gpbs-d10": dict(budget_pct=15, duty=10),
    # hardware samples stall the command processor ~0.2 ms each: the budget
    # is what a sample-hungry mix (frequent switches) pays in tenant time
    "gpbs-b1": dict(budget_pct=1),
    "gpbs-b2": dict(budget_pct=2),
}


class AgreedLoop:
    """Runs ``body`` (one collective) back to back on a thread until stopped.
    Every rank must issue the same number of collectives, but each rank's
    main thread raises its stop at a slightly different moment: a rank that
    starts collective k+1 just before its stop while a peer stopped after k
    would wait in it forever (and so would the join).  The stop is therefore
    agreed on a count: freeze the issue limit at this rank's count, take the
    MAX over ranks (``agree``, e.g. an all-reduce on the ctrl group), and let
    every rank issue up to it before the thread ends."""

    def __init__(self, body: Callable[[], object]):
        self.body = body
        self.cv = threading.Condition()
        self.issued, self.limit, self.stopping = 0, None, False
        self.th = threading.Thread(target=self._run, daemon=True)

    def start(self) -> "AgreedLoop":
        self.th.start()
        return self

    def _run(self):
        while True:
            with self.cv:
                while self.limit is not None and self.issued >= self.limit and not self.stopping:
                    self.cv.wait()
                if self.limit is not None and self.issued >= self.limit:
                    return
                self.issued += 1
            self.body()

    def stop(self, agree: Optional[Callable[[int], int]] = None) -> int:
        """Stop after the agreed count; returns it."""
        with self.cv:
            self.limit = self.issued  # no new collective past this rank's count
            mine = self.issued
        target = max(int(agree(mine)) if agree is not None else mine, mine)
        with self.cv:
            self.limit, self.stopping = target, True
            self.cv.notify_all()
        self.th.join()
        return target


class CollTenant:
    """All-reduce tenant for N > 1: RCCL all-reduce over xGMI on its own
    process group and stream, launch-gated on XCD ownership (RCCL kernels
    themselves are not CU-confined)."""

    def __init__(self, ctx: GpuContext, tenant: int, nbytes: int, group, on_cpu: bool = False,
                 board_name: str = "", rank: int = 0, world: int = 1):
        self.ctx, self.tenant, self.group = ctx, tenant, group
        self.engine: Optional[Engine] = None
        # K10: every all-reduce is timed against the node's arrival board and
        # the wait for the slowest peer goes to the active engine (REPORT_WAIT)
        from ..runtime.waitprobe import ArrivalBoard, WaitProbe
        self.board = ArrivalBoard(board_name, rank, world) if board_name else None
        self.probe = WaitProbe(self._report, board=self.board)
        # on_cpu: bench --rehearse (gloo stand-in for RCCL, all ranks on one GPU)
        self.buf = torch.randn(nbytes // 2, device="cpu" if on_cpu else "cuda",
                               dtype=torch.float32 if on_cpu else torch.bfloat16)
        self.stream = torch.cuda.Stream()
        self.gate = False
        self.units_done = 0
        self.last_done_ns = 0

    def _owns(self):
        return (not self.gate) or self.tenant in self.ctx.owners()

    def run_units(self, n: int):
        import torch.distributed as dist
        if self.engine is not None and self.gate:
            self.engine.wake(self.tenant)
        with torch.cuda.stream(self.stream):
            for _ in range(n):
                while not self._owns():
                    time.sleep(20e-6)
                self.probe.collective(dist.all_reduce, self.buf, group=self.group)
                self.buf.mul_(0.5)
            self.stream.synchronize()
            self.probe.poll()
        self.units_done += n
        self.last_done_ns = time.monotonic_ns()
        if self.engine is not None and self.gate:
            self.engine.block(self.tenant)

    def _report(self, ns: int):
        e = self.engine
        if e is not None:
            try:
                e.report_wait(self.tenant, int(ns))
            except Exception:
                pass

    def close(self):
        if self.board is not None:
            self.board.close()
            self.board = None

    # steady-state protocol: all-reduce back to back until stopped, the stop
    # agreed on a collective count across ranks (AgreedLoop)
    def start_loop(self):
        self._loop = AgreedLoop(lambda: self.run_units(1)).start()

    def stop_loop(self, agree: Optional[Callable[[int], int]] = None):
        self._loop.stop(agree)


def host_cpu_sample() -> Dict[str, float]:
    """This process's CPU time and context switches, and the cgroup's CPU
    throttling (where readable): a run whose launch-bound tenants lose rate
    while the GPU is idle shows here if the host threads were starved."""
    out: Dict[str, float] = {}
    try:
        t = os.times()
        out["cpu_s"] = t.user + t.system
        with open("/proc/self/status") as f:
            for ln in f:
                if ln.startswith(("voluntary_ctxt_switches", "nonvoluntary_ctxt_switches")):
                    k, v = ln.split(":")
                    out[k.strip()] = float(v)
    except OSError:
        pass
    for path in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat"):
        try:
            with open(path) as f:
                for ln in f:
                    k, v = ln.split()
                    if k in ("nr_throttled", "throttled_usec", "throttled_time"):
                        out["cg_" + k] = float(v)
            break
        except (OSError, ValueError):
            continue
    return out


def kfd_queues(pid: Optional[int] = None) -> Optional[int]:
    """Hardware queues KFD holds for a process (sysfs; None where not exposed)."""
    try:
        return len(os.listdir(f"/sys/class/kfd/kfd/proc/{pid or os.getpid()}/queues"))
    except OSError:
        return None


def _pct(xs, q):
    if not xs:
        return 0.0
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))]


class Corun:
    def __init__(self, cfg: CorunConfig, rank: int = 0, world: int = 1, device: int = 0, groups=None, log=print,
                 coll_on_cpu: bool = False):
        self.cfg, self.rank, self.world, self.device = cfg, rank, world, device
        self.coll_on_cpu = coll_on_cpu
        # what this rank's multi-GPU path actually did (bench JSON "ranks")
        self.diag: Dict[str, object] = {"coll": "local" if world == 1 else None, "ipc_selftest": None}
        self.groups = groups or {}
        self.gang = None
        self._gang_seq = 0
        self.gang_stats: Dict[str, float] = {}
        self.log = log if rank == 0 else (lambda *a, **k: None)
        torch.cuda.set_device(device)
        self.engines: Dict[str, Engine] = {}
        self._retired = []  # engines of earlier runs (fresh_engine), closed in close()
        self.tid: Dict[str, int] = {}
        self.tenants = MIXES[cfg.mix]["tenants"]
        self.throughput = MIXES[cfg.mix]["throughput"]
        for pol in cfg.policies:
            if pol in POLICY_ENGINES:
                self.engines[pol] = self._make_engine(pol)
        self.ctx = GpuContext(device, table_mode=cfg.table_mode)
        if not self.tid:  # ids without an engine: fixed order (Domain-0 = 0)
            self.tid = {n: i + 1 for i, (n, _) in enumerate(self.tenants)}
        self.runners: Dict[str, object] = {}
        self.coll_buf = None
        for name, _ in self.tenants:
            self.runners[name] = self._make_runner(name)
        self.quota: Dict[str, int] = {}
        self.solo_unit_ms: Dict[str, float] = {}
        self.solo_est_ms: Dict[str, float] = {}
        self._off: set = set()           # dynamic mix: tenants currently stopped
        self._dyn_t0 = 0
        self._dyn_state: Dict[str, int] = {}
        self.solo_lat_ms = 0.0
        self.active_engine: Optional[Engine] = None
        self._sampler_default = None  # the process's sampler policy (restored after a SAMPLER variant)
        # per-run GPU clock / power / throttle record (pbs_amd/utils/gpustate.py),
        # set by the caller; None: not recorded
        self.gpustate = None

    def _make_runner(self, name: str):
        cfg, t = self.cfg, self.tid[name]
        spec = dict(SPECS[name])
        kind = spec.pop("kind")
        # mem_chunk: unit-boundary granularity of the memory tenants (bytes per
        # work-queue chunk, default 512 KiB) -- how soon a hold or a
        # revocation takes effect
        mem_chunk = {"chunk_bytes": int(cfg.mem_chunk)} if cfg.mem_chunk else {}
        if "alt" in spec and spec["alt"]["kind"] in ("stream", "reduce"):
            spec["alt"] = dict(spec["alt"], **mem_chunk)
        if kind == "gemm":
            return Runner(self.ctx, "gemm", t, depth=cfg.depth, **spec)
        if kind == "stream":
            return Runner(self.ctx, "stream", t, depth=cfg.depth, **spec, **mem_chunk)
        if kind == "reduce":
            if self.world > 1 and cfg.coll_impl == "ipc" and not self.coll_on_cpu:
                r = self._ipc_runner(t, mem_chunk)
                if r is not None:
                    self.diag.update(coll="ipc", ipc_selftest="ok")
                    return r
                self.diag.update(coll="rccl-fallback", ipc_selftest="failed")
                self.log("[corun] IPC all-reduce tenant failed its self-test on this node: using RCCL")
            if self.world > 1:
                if self.diag["coll"] is None:
                    self.diag["coll"] = "gloo-cpu" if self.coll_on_cpu else "rccl"
                return CollTenant(self.ctx, t, cfg.coll_bytes, self.groups.get("coll"), on_cpu=self.coll_on_cpu,
                                  board_name=f"{cfg.gang_shm_base}-arr" if cfg.gang_shm_base else "",
                                  rank=self.rank, world=self.world)
            return Runner(self.ctx, "reduce", t, depth=cfg.depth, bytes=cfg.coll_bytes, **mem_chunk)
        if kind == "gemv":
            return Runner(self.ctx, "gemv", t, depth=1, priority=1, M=cfg.idle_rows, K=cfg.idle_rows)
        raise ValueError(name)

    def _ipc_runner(self, t: int, mem_chunk: dict):
        """The gated IPC all-reduce tenant, after a one-unit self-test on
        every rank: inputs rank + 1, every output element must be the sum
        over ranks (exact in bf16); any rank failing makes all fall back.
        Every step ends in an agreement over the ranks (a MIN of the local
        outcome), so a rank that fails a step never runs ahead into a
        collective its peers are not in."""
        from ..parallel.ipc_coll import IpcColl
        r = None

        def agree(ok: bool) -> bool:
            return -self._allreduce(-(1.0 if ok else 0.0), "max") > 0  # MIN over ranks

        def fail():
            if r is not None:
                r.close()
            if self.coll_buf is not None:
                self.coll_buf.close()
                self.coll_buf = None
            return None
        try:  # the exchanges inside raise on every rank together
            self.coll_buf = IpcColl(self.device, self.rank, self.world, self.cfg.coll_bytes,
                                    group=self.groups.get("ctrl"))
        except Exception as ex:  # noqa: BLE001
            self.log(f"[corun] IPC all-reduce: {ex}")
            self.coll_buf = None
            return None
        ok = True
        try:
            n = self.coll_buf.nbytes // 2
            self.coll_buf.fill(torch.full((n,), float(self.rank + 1), dtype=torch.bfloat16, device="cuda"))
            r = Runner(self.ctx, "allreduce", t, depth=self.cfg.depth, gate=False, engine_wake=False,
                       coll=self.coll_buf, timeout_ms=10000, **mem_chunk)
            torch.cuda.synchronize()
        except Exception as ex:  # noqa: BLE001
            self.log(f"[corun] IPC all-reduce runner: {ex}")
            ok = False
        if not agree(ok):
            return fail()
        try:  # one collective unit on every rank (a P2P-flag barrier inside)
            r.submit(1)
            r.wait(60.0)
            torch.cuda.synchronize()
        except Exception as ex:  # noqa: BLE001
            self.log(f"[corun] IPC all-reduce self-test unit: {ex}")
            ok = False
        if not agree(ok):
            return fail()
        want = float(self.world * (self.world + 1) // 2)
        try:
            good = bool((self.coll_buf.read(1) == want).all().item())
        except Exception:  # noqa: BLE001
            good = False
        if not agree(good):
            return fail()
        g = torch.Generator(device="cuda").manual_seed(4321 + self.rank)
        self.coll_buf.fill(torch.randn(self.coll_buf.nbytes // 2, dtype=torch.bfloat16, device="cuda", generator=g))
        r.set_engine_wake(True)
        r.set_gate(True)
        return r

    def _make_engine(self, pol: str) -> Engine:
        nctx, over, _, table = POLICY_ENGINES[pol]
        prof = {k: v for k, v in MI355X_PROFILE.items()}
        prof.update(over)
        e = Engine(**prof)
        for x in range(8):
            for c in range(nctx):
                e.pool_assign(0, e.partition_add(self.rank, x, c))
        e.tenant_create("Domain-0", nslots=1)
        opts = table.split(",")
        ids = {}
        for name, ns in self.tenants:
            if "budget" in opts:  # one slot per partition; the layout sizes the share
                # (the latency tenant: one per XCD in its lane; a full set as a
                # co-sharer of the region, so the gang leader's runqueue holds it)
                lane = SPECS[name]["kind"] == "gemv" and not MIXES[self.cfg.mix].get("slo_in_region")
                n = ns if lane else XCDS * nctx
            elif "se" in opts:
                n = (SE8_SLOTS if "se8" in opts else SE_SLOTS).get(name, ns if SPECS[name]["kind"] == "gemv" else 16)
            else:
                n = ns
            ids[name] = e.tenant_create(name, nslots=n)
        if self.tid and ids != self.tid:
            raise RuntimeError("tenant ids differ across engines")
        self.tid = ids
        e._gpbs_nctx = nctx
        return e

    # ------------------------------------------------------------- policy
    def _natives(self):
        return [r for r in self.runners.values() if isinstance(r, Runner)]

    def _gang_device(self):
        import torch.distributed as dist
        g = self.groups.get("gang")
        try:
            return f"cuda:{self.device}" if g is not None and dist.get_backend(g) == "nccl" else None
        except Exception:
            return None

    def _stop_gang(self):
        if self.gang is not None:
            self.gang_stats = self.gang.stats()
            self.gang.stop()
            self.gang = None

    def set_policy(self, policy: str):
        self._stop_gang()
        if self.active_engine is not None:
            self.active_engine.stop()
            self.active_engine = None
        coll = self.runners.get("coll")
        if policy in self.engines:
            e = self.engines[policy]
            if self.cfg.fresh_engine and getattr(e, "_gpbs_used", False):
                # the old engine stays alive (closed with the others at the
                # end): the GPU context and runners still reference it until
                # attach() below rebinds them
                self._retired.append(e)
                e = self.engines[policy] = self._make_engine(policy)
            e._gpbs_used = True
            _, _, gate, table = POLICY_ENGINES[policy]
            opts = table.split(",")
            tmode = opts[0]
            try:
                self.ctx.set_table_mode(tmode)
            except RuntimeError as ex:  # no host-accessible fine-grained VRAM pool: the pinned host table
                if tmode != "bar":
                    raise
                self.log(f"[corun] {policy}: {ex}; using the pinned host table")
                self.ctx.set_table_mode("host")
            self.ctx.set_spatial("spatial" in opts)
            self.ctx.set_se_mode("se" in opts)
            self.ctx.set_waveprio("waveprio" in opts)
            self.ctx.set_share("share" in opts)
            self.ctx.set_hold("hold" in opts)
            self.ctx.set_lat_half(1 if "latmem" in opts else -1)
            # device hot path: counter attribution (k_hwc_attribute) and the
            # PBS update (k_adapt) run on the GPU
            # ("hostsched": both on the host -- the bit-exact host twins --
            # so the scheduler puts no kernel on the GPU's queues)
            host_sched = "hostsched" in opts
            self.ctx.attach(e, nctx=e._gpbs_nctx, device_adapt=not host_sched)
            self.ctx.param("device_attr", 0 if host_sched else 1)
            smp = SAMPLER.get(policy)
            if self.cfg.hw_counters and smp != "model":
                if self._sampler_default is None:
                    self._sampler_default = self.ctx.hwc_sampler()
                self.ctx.set_hwc_sampler(**(smp or self._sampler_default))
                self.ctx.set_hwc(True)
            elif self.cfg.hw_counters:
                self.ctx.set_hwc(False)  # modeled counters feed the metric this run
            e.start()
            self.active_engine = e
            in_region = bool(MIXES[self.cfg.mix].get("slo_in_region"))
            for name, r in self.runners.items():
                if not isinstance(r, Runner):
                    continue
                latco = name == "idle" and "latco" in opts and not in_region
                r.set_gate(False if latco else gate)
                r.set_engine_wake(not latco)
            if isinstance(coll, CollTenant):
                coll.gate, coll.engine = True, e
            if self.world > 1 and coll is not None:
                # Cross-GPU gang windows for the all-reduce tenant: its RCCL
                # ranks on all GPUs get their partitions in the same epochs.
                from ..parallel.gang import GangCoordinator
                # own gloo group: the main thread's barriers use "ctrl"
                # The same epochs SUM-reduce the throughput tenants' counters
                # into node-wide metrics (C11).
                self._gang_seq += 1  # same policy order on every rank: same fresh region name
                self._barrier()  # every rank's engine is up before the first gang epoch (no start-up skew)
                tr = self.cfg.gang_transport if self.cfg.gang_shm_base or self.cfg.gang_transport != "shm" else "dist"
                self.gang = GangCoordinator(e, self.groups["gang"], [self.tid["coll"]],
                                            epoch_ms=self.cfg.gang_epoch_ms, share=self.cfg.gang_share,
                                            metric_tenants=[self.tid[n] for n in self.throughput],
                                            transport=tr, rank=self.rank, world=self.world,
                                            shm_name=f"{self.cfg.gang_shm_base}-{self._gang_seq}",
                                            deadline_ms=self.cfg.gang_deadline_ms,
                                            wait_driven=self.cfg.gang_wait_driven,
                                            reform=(tr == "shm"),
                                            device=self._gang_device()).start()
            return
        self.ctx.set_table_mode("host")
        self.ctx.set_spatial(False)
        self.ctx.set_se_mode(False)
        self.ctx.set_share(False)
        self.ctx.set_hold(False)
        self.ctx.set_lat_half(-1)
        self.ctx.set_waveprio(False)
        if self.cfg.hw_counters:
            self.ctx.set_hwc(False)
        for r in self._natives():
            r.set_engine_wake(False)
        if isinstance(coll, CollTenant):
            coll.engine = None
        if policy in ("none", "solo"):
            for r in self._natives():
                r.set_gate(False)
            if isinstance(coll, CollTenant):
                coll.gate = False
        elif policy == "static":  # equal XCD split (ARINC-653-like), tenants in mix order
            order = [n for n, _ in self.tenants]
            per = max(1, 8 // len(order))
            self.ctx.set_owners([self.tid[order[min(x // per, len(order) - 1)]] for x in range(8)])
            for r in self._natives():
                r.set_gate(True)
            if isinstance(coll, CollTenant):
                coll.gate = True
        elif policy in ("static-se", "static-se2"):
            # hand-picked shader-engine layout (STATIC_SE), no engine, no
            # counters: the same SE gating, CU-masked class-half streams and
            # latency tenant (co-resident, raised wave priority) as gpbs
            owners = [-1] * (XCDS * 4)
            for name, (xs, ses) in (STATIC_SE2 if policy == "static-se2" else STATIC_SE)[self.cfg.mix].items():
                for x in xs:
                    for se in ses:
                        owners[x * 4 + se] = self.tid[name]
            self.ctx.set_table_mode("device")
            self.ctx.set_se_mode(True)
            self.ctx.set_waveprio(True)
            self.ctx.set_owners(owners)
            in_region = bool(MIXES[self.cfg.mix].get("slo_in_region"))
            for name, r in self.runners.items():
                if isinstance(r, Runner):
                    r.set_gate(SPECS[name]["kind"] != "gemv" or in_region)
            if isinstance(coll, CollTenant):
                coll.gate = True
        else:
            raise ValueError(policy)

    # ---------------------------------------------------------- primitives
    def _barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier(group=self.groups.get("ctrl"))
        torch.cuda.synchronize()

    def _allreduce(self, v: float, op: str) -> float:
        if self.world == 1:
            return v
        import torch.distributed as dist
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM, group=self.groups.get("ctrl"))
        return float(t.item())

    def _run_units(self, name: str, n: int):
        r = self.runners[name]
        if isinstance(r, Runner):
            r.submit(n)
            r.wait(120.0)
        else:
            r.run_units(n)

    def _collective(self, r) -> bool:
        return isinstance(r, Runner) and r.kind == "allreduce"

    def _drain(self, name: str):
        """Drop a native runner's backlog and let its in-flight units finish;
        the IPC all-reduce tenant stops on a unit count agreed over the ranks
        (its units are collective)."""
        r = self.runners[name]
        if self._collective(r):
            from ..parallel.ipc_coll import agreed_drain
            agreed_drain(r, lambda n: int(self._allreduce(float(n), "max")))
        else:
            r.cancel()
            r.wait(120.0)

    def _estimate_unit_ms(self, name: str) -> float:
        """Rough solo ms per unit (sizes the backlog; not a measurement)."""
        r = self.runners[name]
        self._barrier()
        t0 = time.perf_counter()
        self._run_units(name, 4)
        self._barrier()
        return self._allreduce((time.perf_counter() - t0) * 1e3 / 4, "max")

    def _solo_rate(self, name: str, alt: int, warmup: int, steps: int) -> float:
        """Steady solo rate (units/ms) of one tenant workload: alone on the
        GPU, ungated, backlogged over `warmup` + `steps` windows of step_ms
        -- the same protocol as the co-run, so norm_perf compares like with
        like (slowdown = solo / co-run throughput)."""
        r = self.runners[name]
        step_ns = int(self.cfg.step_ms * 1e6)
        if alt:
            r.set_phase(1)
        if isinstance(r, Runner):
            q = max(1, self.quota.get(name, 16))

            def topup():
                st = r.stats()
                if st.submitted - st.units_done < 2 * q:
                    r.submit(2 * q)
            def done():
                return r.stats().units_done
        else:
            r.start_loop()

            def topup():
                pass
            def done():
                return r.units_done
        self._barrier()
        t0 = d0 = None
        for w in range(warmup + steps):
            if w == warmup:
                t0, d0 = time.perf_counter(), done()
            end = time.monotonic_ns() + step_ns
            while time.monotonic_ns() < end:
                topup()
                time.sleep(5e-4)
        dt_ms = (time.perf_counter() - t0) * 1e3
        rate = (done() - d0) / dt_ms
        if isinstance(r, Runner):
            self._drain(name)
        else:
            r.stop_loop(agree=lambda n: int(self._allreduce(float(n), "max")))
        if alt:
            r.set_phase(0)
        self._barrier()
        return -self._allreduce(-rate, "max")  # min over ranks

    def calibrate(self):
        """Solo rate of every throughput tenant -- and of each workload of a
        phase-changing tenant -- under the steady protocol (W warmup + K timed
        windows, backlogged, alone, ungated), and the latency tenant's solo p50."""
        self.set_policy("solo")
        cfg = self.cfg
        steps = cfg.solo_steps or cfg.steps
        for name in self.throughput:
            r = self.runners[name]
            kinds = (0, 1) if getattr(r, "alt_kind", None) else (0,)
            for alt in kinds:
                key = f"{name}:alt" if alt else name
                if alt:
                    r.set_phase(1)
                est = self._estimate_unit_ms(name)
                if alt:
                    r.set_phase(0)
                self.quota[key] = max(1, int(round(cfg.target_ms / est)))
                self.quota[name] = max(self.quota.get(name, 1), self.quota[key])
                rate = self._solo_rate(name, alt, cfg.warmup, steps)
                self.solo_unit_ms[key] = 1.0 / rate if rate > 0 else est
                self.solo_est_ms[key] = est
        r = self.runners.get("idle")
        if r is not None:
            r.latencies(clear=True)
            for _ in range(20):
                r.submit(1)
                r.wait(10.0)
                time.sleep(cfg.idle_period_ms / 1e3)
            self.solo_lat_ms = _pct(r.latencies(clear=True), 0.5) / 1e6
        self.log(f"[corun] solo unit ms (steady): {self.solo_unit_ms}  (round-trip estimate {self.solo_est_ms})  "
                 f"quota/step: {self.quota}  idle p50 {self.solo_lat_ms:.3f} ms")

    def solo_report(self) -> Dict[str, Dict]:
        """Solo rates with the workload's physical rate (TF/s, TB/s) for a
        check against scripts/kbench.py."""
        out = {}
        for key, ms in self.solo_unit_ms.items():
            name, alt = key.split(":")[0], key.endswith(":alt")
            r = self.runners[name]
            d = {"solo_units_per_ms": round(1.0 / ms, 4), "solo_unit_ms": round(ms, 5),
                 "roundtrip_estimate_unit_ms": round(self.solo_est_ms.get(key, 0.0), 5)}
            if isinstance(r, Runner):
                work = r.alt_work_per_unit if alt else r.work_per_unit
                kind = r.alt_kind if alt else r.kind
                if kind == "gemm":
                    d["solo_tflops"] = round(work / (ms * 1e-3) / 1e12, 1)
                else:
                    d["solo_tbps"] = round(work / (ms * 1e-3) / 1e12, 3)
            out[key] = d
        return out

    def step(self) -> Dict[str, float]:
        """One co-run step; returns per-tenant completion times (ms) in the step."""
        cfg = self.cfg
        t0 = time.monotonic_ns()
        threads = []
        target = {}
        for name in self.throughput:
            r = self.runners[name]
            if isinstance(r, Runner):
                target[name] = r.stats().units_done + self.quota[name]
                r.submit(self.quota[name])
            else:
                th = threading.Thread(target=r.run_units, args=(self.quota[name],))
                th.start()
                threads.append(th)
        idle = self.runners.get("idle")
        nreq = 0
        while True:  # latency tenant: closed loop with think time while others run
            if idle is not None:
                idle.submit(1)
                idle.wait(30.0)
                nreq += 1
            busy = any(self.runners[n].stats().units_done < target[n] for n in target) or \
                any(t.is_alive() for t in threads)
            if not busy:
                break
            time.sleep(cfg.idle_period_ms / 1e3 if idle is not None else 2e-4)
        for name in target:
            self.runners[name].wait(120.0)
        for th in threads:
            th.join()
        done = {}
        for name in self.throughput:
            r = self.runners[name]
            last = r.stats().last_done_ns if isinstance(r, Runner) else r.last_done_ns
            done[name] = (last - t0) / 1e6
        done["_step"] = (time.monotonic_ns() - t0) / 1e6
        done["_nreq"] = nreq
        return done

    def _done(self, name: str) -> int:
        r = self.runners[name]
        return r.stats().units_done if isinstance(r, Runner) else r.units_done

    def _dyn_apply(self):
        """Mix "phase": the phase tenant's workload and the hbm tenant's
        presence follow a fixed schedule from the start of the run (warmup
        included), the same for every policy."""
        if not MIXES[self.cfg.mix].get("dynamic"):
            return
        el = (time.monotonic_ns() - self._dyn_t0) / 1e6
        want = {"phase": int(el // self.cfg.phase_ms) % 2, "hbm": int(el // self.cfg.onoff_ms) % 2 == 0}
        if self._dyn_state.get("phase") != want["phase"]:
            self.runners["phase"].set_phase(want["phase"])
            self._dyn_state["phase"] = want["phase"]
            self._dyn_state["flips"] = self._dyn_state.get("flips", 0) + 1
        if self._dyn_state.get("hbm") != want["hbm"]:
            self._dyn_state["hbm"] = want["hbm"]
            if want["hbm"]:
                self._off.discard("hbm")
            else:
                self._off.add("hbm")
                self.runners["hbm"].cancel()  # drains its in-flight units, then blocks its slots

    def _dyn_reset(self):
        if MIXES[self.cfg.mix].get("dynamic"):
            self.runners["phase"].set_phase(0)
        self._off.clear()
        self._dyn_state = {}

    def _idle_request(self, until_ns: int):
        """Latency tenant: closed loop with think time until `until_ns`."""
        idle = self.runners.get("idle")
        n = 0
        while time.monotonic_ns() < until_ns:
            self._dyn_apply()
            if idle is not None:
                idle.submit(1)
                idle.wait(30.0)
                n += 1
            self._topup()
            time.sleep(self.cfg.idle_period_ms / 1e3 if idle is not None else 2e-4)
        return n

    def _topup(self):
        """Keep every native throughput runner backlogged (>= 2 quotas queued)."""
        for name in self.throughput:
            if name in self._off:
                continue
            r = self.runners[name]
            if isinstance(r, Runner):
                st = r.stats()
                if st.submitted - st.units_done < 2 * self.quota[name]:
                    r.submit(2 * self.quota[name])

    def _work(self, name: str):
        """(units done, of which alternate-workload units)."""
        r = self.runners[name]
        if isinstance(r, Runner):
            st = r.stats()
            return st.units_done, st.units_alt
        return r.units_done, 0

    def _solo_equiv(self, name: str, du: int, da: int) -> float:
        """Solo-time equivalent (ms) of du units, da of them alternate-workload."""
        ms = self.solo_unit_ms[name]
        return (du - da) * ms + da * self.solo_unit_ms.get(f"{name}:alt", ms)

    def run_policy_steady(self, policy: str, steps: int, warmup: int) -> Dict:
        """Steady-state weighted speedup: all throughput tenants backlogged for
        W + K windows of step_ms; the K timed windows give each tenant's
        co-run throughput (units / ms), normalised by its solo rate."""
        self.set_policy(policy)
        cfg = self.cfg
        coll = self.runners.get("coll")
        self._dyn_state = {}
        self._dyn_t0 = time.monotonic_ns()
        self._dyn_apply()
        self._topup()
        if isinstance(coll, CollTenant):
            coll.start_loop()
        step_ns = int(cfg.step_ms * 1e6)
        for _ in range(warmup):
            self._idle_request(time.monotonic_ns() + step_ns)
        if "idle" in self.runners:
            self.runners["idle"].latencies(clear=True)
        for n in self.tid:
            self.ctx.ownership(self.tid[n], clear=True)
        e = self.active_engine
        if e is not None:
            e.perfc_reset()
            run0 = {n: e.tenant_info(self.tid[n]).run_ns for n in self.tid}
            for n in self.throughput:
                e.bound_stats(self.tid[n], reset=True)
            if self.cfg.hw_counters:
                self.ctx.hwc_reset()
        quanta = {n: [] for n in self.tid}
        self._targets = {n: [] for n in self.tid}  # the policy's target quantum per step (PBS: adaptive)
        layout = {n: [] for n in self.throughput}  # budget SE sets per step (bit c = SE c)
        self._rs0 = {n: r.stats() for n, r in self.runners.items() if isinstance(r, Runner)}
        self.ctx.masked_pool_reset()
        _gs0 = self.ctx.stats()  # the pool's counters are process-wide: this run's share is the delta
        if self.cfg.kernel_trace:
            from ..counters import hwc as _hwc
            _hwc.trace_stats(reset=True)
        self._barrier()
        t0 = time.perf_counter()
        g0 = time.monotonic()
        h0 = host_cpu_sample()
        d0 = {n: self._work(n) for n in self.throughput}
        per_step = []
        for _ in range(steps):
            ts, ds = time.perf_counter(), {n: self._work(n) for n in self.throughput}
            self._idle_request(time.monotonic_ns() + step_ns)
            te = time.perf_counter()
            dn = {n: self._work(n) for n in self.throughput}
            per_step.append({n: self._solo_equiv(n, dn[n][0] - ds[n][0], dn[n][1] - ds[n][1]) / ((te - ts) * 1e3)
                             for n in self.throughput})
            if e is not None:
                for n in self.tid:
                    ti = e.tenant_info(self.tid[n])
                    quanta[n].append(ti.tslice_us)  # dispatched (s_timer) quantum
                    self._targets[n].append(ti.target_tslice_us)
                    if n in layout:
                        layout[n].append(ti.budget_ctx)
        d1 = {n: self._work(n) for n in self.throughput}
        wall_ms_local = (time.perf_counter() - t0) * 1e3
        g1 = time.monotonic()
        h1 = host_cpu_sample()
        self._barrier()
        wall_ms = self._allreduce(wall_ms_local, "max")
        # drain: drop the backlog, let in-flight units finish
        for name in self.throughput:
            r = self.runners[name]
            if isinstance(r, Runner) and not self._collective(r):
                r.cancel()
        if isinstance(coll, CollTenant):
            coll.stop_loop(agree=lambda n: int(self._allreduce(float(n), "max")))
        for name in self.throughput:
            r = self.runners[name]
            if isinstance(r, Runner):
                if self._collective(r):
                    self._drain(name)
                else:
                    r.wait(120.0)
        flips = self._dyn_state.get("flips", 0)
        self._dyn_reset()
        lats = [x / 1e6 for x in self.runners["idle"].latencies(clear=True)] if "idle" in self.runners else []
        res = {"policy": policy, "protocol": "steady", "wall_ms": wall_ms, "ms_per_step": wall_ms / steps,
               "tenants": {}}
        if MIXES[cfg.mix].get("dynamic"):
            res["phase_flips"] = flips
        if self.gpustate is not None:  # the GPU's clock / power / throttle state over the timed window
            res["gpu_state"] = self.gpustate.window(g0, g1)
        nq = kfd_queues()
        if nq is not None:  # hardware queues this process holds (KFD): oversubscription shows here
            res["kfd_queues"] = nq
        # CU-masked queues held at once over the run and acquires that had to
        # share another layout's queue (serialised layouts)
        gs = self.ctx.stats()
        res["masked_queues"] = {"held_max": gs["masked_queues_held_max"], "created": gs["masked_queues_created"],
                                "cross_key_shares": gs["masked_cross_key_shares"] - _gs0["masked_cross_key_shares"],
                                "pipe_shared_other": gs["masked_pipe_shared_other"] - _gs0["masked_pipe_shared_other"]}
        if self.cfg.kernel_trace:  # in-process kernel trace of the run (live counters on)
            from ..counters import hwc as _hwc
            ks = _hwc.trace_stats(reset=True)
            if ks:
                res["kernel_trace"] = ks
        res["host"] = {k: round(h1[k] - h0[k], 3) for k in h1 if k in h0}
        if "cpu_s" in res["host"]:
            res["host"]["cpu_util"] = round(res["host"]["cpu_s"] / (wall_ms_local / 1e3), 2)  # cores busy
        agg, slows = 0.0, []
        for n in self.throughput:
            du, da = d1[n][0] - d0[n][0], d1[n][1] - d0[n][1]
            rate = du / wall_ms_local  # units per ms
            perf = self._solo_equiv(n, du, da) / wall_ms_local
            agg += perf
            slows.append((1.0 / perf - 1.0) * 100.0 if perf > 0 else 1e4)
            res["tenants"][n] = {"units": du, "units_per_ms": round(rate, 4),
                                 "solo_units_per_ms": round(1.0 / self.solo_unit_ms[n], 4),
                                 "norm_perf": round(perf, 4), "slowdown_pct": round(slows[-1], 2),
                                 "step_norm_perf": [round(ps[n], 3) for ps in per_step]}
            if da:
                res["tenants"][n]["units_alt"] = da
            if e is not None and any(layout[n]):
                res["tenants"][n]["se_layout"] = layout[n]
        self._finish_result(res, e, lats, slows, agg, wall_ms, quanta, run0 if e is not None else None, policy)
        self.log(f"[corun] {policy}: " + json.dumps(res))
        return res

    def run_policy(self, policy: str, steps: int, warmup: int) -> Dict:
        from ..utils import roctx
        with roctx.range(f"gpbs:policy {policy}"):
            return self._run_policy(policy, steps, warmup)

    def _run_policy(self, policy: str, steps: int, warmup: int) -> Dict:
        if self.cfg.protocol == "steady":
            return self.run_policy_steady(policy, steps, warmup)
        self.set_policy(policy)
        for _ in range(warmup):
            self.step()
        if "idle" in self.runners:
            self.runners["idle"].latencies(clear=True)
        for n in self.tid:
            self.ctx.ownership(self.tid[n], clear=True)
        e = self.active_engine
        if e is not None:
            e.perfc_reset()
            run0 = {n: e.tenant_info(self.tid[n]).run_ns for n in self.tid}
            if self.cfg.hw_counters:
                self.ctx.hwc_reset()
        per = {n: [] for n in self.throughput}
        self._barrier()
        t0 = time.perf_counter()
        quanta = {n: [] for n in self.tid}
        for _ in range(steps):
            d = self.step()
            for n in self.throughput:
                per[n].append(d[n])
            if e is not None:
                for n in self.tid:
                    quanta[n].append(e.tenant_info(self.tid[n]).tslice_us)
        self._barrier()
        wall_ms = self._allreduce((time.perf_counter() - t0) * 1e3, "max")
        lats = [x / 1e6 for x in self.runners["idle"].latencies(clear=True)] if "idle" in self.runners else []
        res = {"policy": policy, "wall_ms": wall_ms, "ms_per_step": wall_ms / steps, "tenants": {}}
        agg = 0.0
        slows = []
        for n in self.throughput:
            t_i = statistics.mean(per[n])
            T_i = self.quota[n] * self.solo_unit_ms[n]
            perf = T_i / t_i if t_i > 0 else 0.0
            agg += perf
            slows.append((t_i / T_i - 1.0) * 100.0)
            res["tenants"][n] = {"corun_ms": round(t_i, 3), "solo_ms": round(T_i, 3), "norm_perf": round(perf, 4),
                                 "slowdown_pct": round(slows[-1], 2)}
        self._finish_result(res, e, lats, slows, agg, wall_ms, quanta, run0 if e is not None else None, policy)
        self.log(f"[corun] {policy}: " + json.dumps(res))
        return res

    def _finish_result(self, res, e, lats, slows, agg, wall_ms, quanta, run0, policy):
        p50, p99 = _pct(lats, 0.5), _pct(lats, 0.99)
        idle_perf = self.solo_lat_ms / p50 if p50 > 0 else 0.0
        if "idle" in self.runners:
            slows.append((p50 / self.solo_lat_ms - 1.0) * 100.0 if self.solo_lat_ms > 0 else 0.0)
            res["tenants"]["idle"] = {"p50_ms": round(p50, 4), "p99_ms": round(p99, 4),
                                      "solo_p50_ms": round(self.solo_lat_ms, 4), "norm_perf": round(idle_perf, 4),
                                      "slowdown_pct": round(slows[-1], 2), "requests": len(lats),
                                      "over_ms": {str(b): sum(1 for x in lats if x > b) for b in (0.5, 1, 2, 5)}}
        res["aggregate"] = agg
        res["aggregate_all_gpus"] = self._allreduce(agg, "sum")
        res["mean_slowdown_pct"] = statistics.mean(slows)
        if e is not None:
            pc = e.perfc()
            eng = {k: pc[k] for k in ("sched_ctx", "acct_run", "metric_tick", "adapt_inc", "adapt_dec",
                                      "adapt_rearm", "migrate_queued", "vcpu_wake_runnable", "tickle_idlers_some",
                                      "class_change", "relayout")}
            eng["gpu"] = self.ctx.stats()
            if self.cfg.hw_counters and SAMPLER.get(policy) != "model":
                eng["hwc"] = self.ctx.hwc_stats()
                eng["hwc"]["share_frac"] = round(self.ctx.share_ns() / (wall_ms * 1e6), 4)
                # Hardware-derived PBS metrics per tenant over the timed window
                # (ownership-attributed counts): L2 misses and L2 requests per
                # 100k instructions, cycles per 1k instructions.
                hw = {}
                for n in self.tid:
                    att, mod = self.ctx.hwc_tenant(self.tid[n])
                    inst = att[0]
                    hw[n] = {"inst": round(inst), "miss_rate": round(att[3] * 1e5 / inst) if inst else 0,
                             "l2_req_rate": round(att[2] * 1e5 / inst) if inst else 0,
                             "cpi_x1000": round(att[1] * 1e3 / inst) if inst else 0,
                             "model_miss_rate": round(mod[3] * 1e5 / mod[0]) if mod[0] else 0}
                eng["hw_tenant"] = hw
                # per throughput tenant: metric periods from a clean hardware
                # window vs the calibrated modeled fallback (and skipped ones)
                per = {n: self.ctx.hwc_tenant_periods(self.tid[n]) for n in self.throughput}
                eng["hwc"]["tenant_periods"] = per
                frac = {}
                for n, v in per.items():
                    m = v["clean"] + v["fallback"]
                    frac[n] = round(v["clean"] / m, 3) if m else 0.0
                eng["hwc"]["per_tenant_clean_frac"] = frac
            eng["miss_rate"] = {n: e.tenant_info(self.tid[n]).cache_miss_rate for n in self.tid}
            eng["class"] = {n: e.lib.gpbs_tenant_class(e.h, self.tid[n]) for n in self.tid}
            eng["mean_tslice_us"] = {n: round(statistics.mean(q), 1) for n, q in quanta.items() if q}  # dispatched
            tg = getattr(self, "_targets", {})
            eng["mean_target_tslice_us"] = {n: round(statistics.mean(q), 1) for n, q in tg.items() if q}
            # measured switch costs (drain + ramp) and the engine's floor basis
            eng["switch_cost"] = {n: dict(self.ctx.switch_cost(self.tid[n]),
                                          engine_us=e.tenant_info(self.tid[n]).switch_cost_us)
                                  for n in self.tid}
            eng["shared"] = {n: e.tenant_info(self.tid[n]).budget_shared for n in self.tid}
            eng["budget_ctx"] = {n: e.tenant_info(self.tid[n]).budget_ctx for n in self.tid}
            eng["online"] = {n: e.tenant_info(self.tid[n]).online_slots for n in self.tid}
            eng["perfc"] = {k: v for k, v in e.perfc().items()
                            if k in ("relayout", "probe_layout", "probe_expired", "class_change")}
            # measured metric periods and, of those, at the quantum bounds
            eng["at_bound"] = {n: e.bound_stats(self.tid[n]) for n in self.throughput}
            eng["measure_tenures"] = {n: e.measure(self.tid[n]) for n in self.throughput}
            eng["run_share"] = {n: round((e.tenant_info(self.tid[n]).run_ns - run0[n]) / (wall_ms * 1e6), 3)
                                for n in self.tid}
            eng["phase"] = {n: e.tenant_info(self.tid[n]).phase for n in self.tid}
            eng["ctx_share"] = {n: [round(x / (wall_ms / 1e3), 2) for x in self.ctx.ownership(self.tid[n])]
                                for n in self.tid}
            eng["runner"] = {}
            rs0 = getattr(self, "_rs0", {})
            for n, r in self.runners.items():
                if not isinstance(r, Runner):
                    continue
                st, s0 = r.stats(), rs0.get(n)
                d = {k: getattr(st, k) - (getattr(s0, k) if s0 else 0)
                     for k in ("launches", "relaunches", "waits_owner", "drain_count", "drain_sum_ns")}
                # revocation drain: table publish -> the interrupted unit's grid gone
                d["drain_us_mean"] = round(d.pop("drain_sum_ns") / d["drain_count"] / 1e3, 1) if d["drain_count"] else None
                d["queue"] = r.queue_index()  # which masked queue (hardware pipe) the run ended on
                eng["runner"][n] = d
            eng["hold_raises"] = self.ctx.hold_raises()  # latency-request holds (cumulative, gpbs-lat)
            coll = self.runners.get("coll")
            if isinstance(coll, CollTenant):
                eng["coll_wait"] = coll.probe.stats()  # K10 reports (cumulative)
            if self.gang is not None:
                eng["gang"] = self.gang.stats()
                names = {v: k for k, v in self.tid.items()}
                eng["node_metrics"] = {names.get(t, t): m for t, m in self.gang.node_metrics.items()}
                eng["node_totals"] = {names.get(t, t): m for t, m in self.gang.node_totals.items()}
            res["engine"] = eng
            diag = os.environ.get("GPBS_DIAG_DIR")
            if diag and self.rank == 0:
                os.makedirs(diag, exist_ok=True)
                import gzip
                recs = e.trace(max_records=1 << 16, from_start=False)
                self._diag_n = getattr(self, "_diag_n", 0) + 1
                with gzip.open(os.path.join(diag, f"trace_{policy}_{self._diag_n:02d}.json.gz"), "wt") as f:
                    json.dump({"tid": self.tid, "lat_ms": lats, "aggregate": agg, "engine": eng,
                               "trace": [[r.t_ns, r.event, r.cpu, *r.a] for r in recs]}, f)

    def close(self):
        self._stop_gang()
        if self.active_engine is not None:
            self.active_engine.stop()
        for r in self._natives():
            r.close()
        if self.coll_buf is not None:
            self.coll_buf.close()
            self.coll_buf = None
        coll = self.runners.get("coll")
        if isinstance(coll, CollTenant):
            coll.close()
        self.ctx.close()
        for e in list(self.engines.values()) + self._retired:
            e.close()
