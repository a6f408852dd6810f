"""gpbsd: the node-level scheduler daemon.

Owns one native engine whose partitions are the (GPU, XCD, issue-context)
triples of the node, the tenant control-page region (+ bridge thread), and
the Unix-socket RPC server that gpbsctl / libgpbs clients talk to (the
toolstack -> hypercall path of the reference: X:tools/libxl/xl_cmdimpl.c ->
libxl -> libxc -> privcmd -> domctl/sysctl).

    python -m pbs_amd.runtime.daemon --socket /tmp/gpbsd.sock --gpus 0 [--sim] [--config gpbs.toml]

Snapshots: scheduler state (pools, tenants, weights/caps, pins, PBS windows)
is written to ``--state`` on SIGTERM and every ``--snapshot-s`` seconds, and
restored at start-up when the file exists.
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import signal
import sys
import threading
import time
from typing import Any, Dict, List, Optional

from .. import _native as N
from ..core import config as cfgmod
from ..core.engine import PMC_NAMES, Engine
from ..ctl.rpc import DEFAULT_SOCKET, RpcError, Server
from ..utils import snapshot as snap

XCDS = 8


class Daemon:
    _seq = 0

    def __init__(self, socket_path: str = DEFAULT_SOCKET, gpus=(0,), nctx: int = 2, sim: bool = False,
                 profile: str = "mi355x", config_path: Optional[str] = None, ctl_name: str = "gpbs",
                 ctl_pages: int = 64, state_path: Optional[str] = None, attach_gpu: bool = False,
                 overrides: Optional[Dict[str, Any]] = None, se_mode: bool = False, hw_counters: bool = False):
        prof = cfgmod.MI355X_PROFILE if profile == "mi355x" else cfgmod.REFERENCE_PROFILE
        self.cfg = cfgmod.load(config_path or os.environ.get("GPBS_CONFIG") or None, prof)
        kw = cfgmod.engine_kwargs(self.cfg)
        kw.update(overrides or {})
        kw["sim_clock"] = int(sim)
        # se_mode: the nctx(=4) partitions of an XCD are its shader engines,
        # owned exclusively; torch tenants run on streams masked to the SEs
        # they own, so the per-SE hardware counters (hw_counters; needs
        # pbs_amd.counters.hwc.init() before HIP init and hwc.start()) are
        # attributed to them by ownership -- measured, not declared.
        self.se_mode = bool(se_mode)
        self.hw_counters = bool(hw_counters)
        self.engine = Engine(**kw)
        self.gpus = list(gpus)
        self.nctx = nctx
        self.part_of: Dict[tuple, int] = {}
        for g in self.gpus:
            for x in range(XCDS):
                for c in range(nctx):
                    pid = self.engine.partition_add(g, x, c)
                    self.part_of[(g, x, c)] = pid
                    self.engine.pool_assign(0, pid)
        self.dom0 = self.engine.tenant_create("Domain-0", nslots=1)
        self.lib = N.load_core()
        Daemon._seq += 1
        self.ctl_name = f"{ctl_name}-{os.getpid()}-{Daemon._seq}"
        self.ctl = self.lib.gpbs_ctl_create(self.ctl_name.encode(), ctl_pages)
        if not self.ctl:
            raise RuntimeError("cannot create control-page region")
        self.ctl = C.c_void_p(self.ctl)
        self.pages: Dict[int, int] = {}  # tenant -> page
        self.pids: Dict[int, int] = {}   # tenant -> registered process
        self.reaped: List[str] = []
        self.gpu_ctx = None
        self.gpu_ctxs: List[Any] = []
        if attach_gpu:
            self.attach_backends(self._gpu_backend)
        self.lib.gpbs_ctl_bind(self.ctl, self.engine.h)
        self.state_path = state_path
        self.lock = threading.RLock()
        self._apply_config()
        if state_path and os.path.exists(state_path):
            self.restore(state_path)
        self.socket_path = socket_path
        self.server = Server(socket_path, self._handlers())
        self.sim = sim
        self.running = False

    # ------------------------------------------------------ GPU backends
    def _gpu_backend(self, gpu: int, part_lo: int):
        from .gpu import GpuContext
        ctx = GpuContext(gpu, part_base=part_lo, nctx=self.nctx, params=self.cfg.get("runtime", {}))
        ctx.attach_mux(self.engine, nctx=self.nctx)
        if self.se_mode:
            # the partition table in BAR-written VRAM: switches put no kernel
            # on the GPU (the pinned host table where no such pool exists)
            try:
                ctx.set_table_mode("bar")
            except RuntimeError:
                pass
            ctx.set_se_mode(True, pool=False)  # the tenants are other processes
        if self.hw_counters:
            from ..counters import hwc
            if not hwc.active():
                hwc.start()  # after HIP init (the GpuContext above), once per process
            ctx.set_hwc(True)
        return ctx

    def attach_backends(self, factory):
        """One actuator + counter backend per managed GPU.  ``factory(gpu,
        part_lo)`` builds it and registers it on the engine's backend mux for
        the GPU's partitions [part_lo, part_lo + 8 * nctx) (a GpuContext on a
        GPU box; a fake in CPU tests).  Partitions of every GPU are driven --
        the engine spans the node."""
        for g in self.gpus:
            b = factory(g, self.part_of[(g, 0, 0)])
            self.gpu_ctxs.append(b)
        self.gpu_ctx = self.gpu_ctxs[0] if self.gpu_ctxs else None
        return self.gpu_ctxs

    # ----------------------------------------------------------- helpers
    def _resolve(self, dom) -> int:
        if isinstance(dom, int) or (isinstance(dom, str) and dom.lstrip("-").isdigit()):
            t = int(dom)
            if t not in self.engine.tenants():
                raise RpcError(f"Domain '{dom}' does not exist.", -2)
            return t
        try:
            return self.engine.tenant_find(str(dom))
        except Exception:
            raise RpcError(f"Domain '{dom}' does not exist.", -2)

    def _pool(self, pool) -> int:
        if pool is None:
            return 0
        if isinstance(pool, int) or (isinstance(pool, str) and pool.isdigit()):
            p = int(pool)
            if p not in self.engine.pools():
                raise RpcError(f"unknown cpupool '{pool}'", -2)
            return p
        try:
            return self.engine.pool_find(str(pool))
        except Exception:
            raise RpcError(f"unknown cpupool '{pool}'", -2)

    def _cpus_arg(self, spec) -> List[int]:
        """'3', '0-5,9', 'node:1' (all partitions of GPU 1), 'gpu1:xcd2' or 'all'."""
        n = self.engine.num_partitions
        if spec in (None, "all"):
            return list(range(n))
        out: List[int] = []
        for part in str(spec).split(","):
            part = part.strip()
            if part.startswith("node:") or part.startswith("gpu:"):
                g = int(part.split(":")[1])
                out += [p for (gg, x, c), p in self.part_of.items() if gg == g]
            elif part.startswith("gpu") and ":xcd" in part:
                g, x = part[3:].split(":xcd")
                out += [p for (gg, xx, c), p in self.part_of.items() if gg == int(g) and xx == int(x)]
            elif "-" in part:
                a, b = part.split("-")
                out += list(range(int(a), int(b) + 1))
            else:
                out.append(int(part))
        return sorted(set(out))

    def _apply_config(self):
        for name, pc in self.cfg.get("pools", {}).items():
            pid = self.engine.pool_create(name, pc.get("sched", ""))
            for p in self._cpus_arg(pc.get("cpus", "")) if pc.get("cpus") else []:
                owner = self.engine.partition_info(p)["pool"]
                if owner >= 0:
                    self.engine.pool_unassign(owner, p)
                self.engine.pool_assign(pid, p)
        for name, tc in self.cfg.get("tenants", {}).items():
            self.create(name=name, slots=int(tc.get("slots", tc.get("vcpus", 8))),
                        weight=int(tc.get("weight", tc.get("cpu_weight", -1))), cap=int(tc.get("cap", -1)),
                        pool=tc.get("pool"))

    # ------------------------------------------------------------ methods
    def info(self):
        return {"version": 1, "abi": self.lib.gpbs_abi_version(), "gpus": self.gpus, "nctx": self.nctx,
                "partitions": self.engine.num_partitions, "pools": self.pool_list(), "ctl": self.ctl_name,
                "sim": self.sim}

    def create(self, name: str, slots: int = 8, weight: int = -1, cap: int = -1, pool=None):
        with self.lock:
            return self.engine.tenant_create(name, nslots=slots, pool=self._pool(pool), weight=weight, cap=cap)

    def destroy(self, domain):
        with self.lock:
            t = self._resolve(domain)
            if t == self.dom0:
                raise RpcError("cannot destroy Domain-0", -22)
            self.engine.tenant_destroy(t)
            page = self.pages.pop(t, None)
            if page is not None:
                self.lib.gpbs_ctl_assign(self.ctl, page, -1)
            self.pids.pop(t, None)
            return 0

    def domain_list(self):
        out = []
        for t in self.engine.tenants():
            i = self.engine.tenant_info(t)
            out.append({"id": t, "name": i.name, "pool": i.pool, "weight": i.weight, "cap": i.cap,
                        "slots": i.nslots, "paused": i.paused, "tslice_us": i.tslice_us, "phase": i.phase,
                        "miss_rate": i.cache_miss_rate, "run_ns": i.run_ns})
        return out

    def domain_sched_get(self, domain):
        t = self._resolve(domain)
        w, c = self.engine.sched_credit_get(t)
        return {"id": t, "name": self.engine.tenant_info(t).name, "weight": w, "cap": c}

    def domain_sched_set(self, domain, weight: int = -1, cap: int = -1):
        with self.lock:
            t = self._resolve(domain)
            self.engine.sched_credit_set(t, weight, cap)
            return self.domain_sched_get(t)

    def domain_sched_ext_get(self, domain):
        """xl sched-credit2 / sched-sedf -d: scheduler-specific parameters."""
        t = self._resolve(domain)
        x = self.engine.sched_ext_get(t)
        i = self.engine.tenant_info(t)
        x.update({"id": t, "name": i.name, "pool": i.pool, "sched": self.engine.pool_info(i.pool)["sched"]})
        return x

    def domain_sched_ext_set(self, domain, weight: int = 0, period_us: int = 0, slice_us: int = 0,
                             latency_us: int = -1, extratime: int = -1):
        with self.lock:
            t = self._resolve(domain)
            self.engine.sched_ext_set(t, weight=int(weight), period_us=int(period_us), slice_us=int(slice_us),
                                      latency_us=int(latency_us), extratime=int(extratime))
            return self.domain_sched_ext_get(t)

    def pool_params_get(self, pool=None):
        p = self._pool(pool)
        ts, rl = self.engine.sched_params_get(p)
        return {"pool": p, "name": self.engine.pool_info(p)["name"], "tslice_us": ts, "ratelimit_us": rl}

    def pool_params_set(self, pool=None, tslice_us: Optional[int] = None, ratelimit_us: Optional[int] = None):
        with self.lock:
            p = self._pool(pool)
            ts, rl = self.engine.sched_params_get(p)
            ts = ts if tslice_us is None else int(tslice_us)
            rl = rl if ratelimit_us is None else int(ratelimit_us)
            # libxl validation (libxl.c:4081-4101), with messages
            if ts < cfgmod_min_tslice() or ts > 1000000:
                raise RpcError(f"Time slice out of range, valid range is from {cfgmod_min_tslice()} to 1000000", -22)
            if rl < 100 or rl > 500000:
                raise RpcError("Ratelimit out of range, valid range is from 100 to 500000", -22)
            if rl > ts:
                raise RpcError("Ratelimit cannot be greater than timeslice", -22)
            self.engine.sched_params_set(p, ts, rl)
            return self.pool_params_get(p)

    def arinc653_get(self, pool=None):
        p = self._pool(pool)
        try:
            s = self.engine.arinc653_get(p)
        except Exception:
            raise RpcError("Pool is not using the arinc653 scheduler", -22)
        names = {}
        for t in self.engine.tenants():
            names[t] = self.engine.tenant_info(t).name
        s["entries"] = [{"domain": names.get(t, str(t)), "id": t, "slot": sl, "runtime_us": rt}
                        for t, sl, rt in s["entries"]]
        s.update(pool=p, name=self.engine.pool_info(p)["name"])
        return s

    def arinc653_set(self, pool=None, major_frame_us: float = 0, entries=()):
        """entries: [{"domain": name|id, "slot": -1|k, "runtime_us": us}, ...]."""
        with self.lock:
            p = self._pool(pool)
            es = [(self._resolve(x["domain"]), int(x.get("slot", -1)), float(x["runtime_us"])) for x in entries]
            if not es:
                raise RpcError("Schedule must have at least one entry", -22)
            if float(major_frame_us) <= 0:
                raise RpcError("Major frame must be positive", -22)
            if sum(x[2] for x in es) > float(major_frame_us):
                raise RpcError("Total runtime of the entries exceeds the major frame", -22)
            try:
                self.engine.arinc653_set(p, float(major_frame_us), es)
            except Exception as e:
                raise RpcError(f"Invalid ARINC 653 schedule: {e}", -22)
            return self.arinc653_get(p)

    def pool_list(self):
        out = []
        for p in self.engine.pools():
            info = self.engine.pool_info(p)
            out.append(info)
        return out

    def pool_create(self, name: str, sched: str = "credit", cpus=None):
        with self.lock:
            pid = self.engine.pool_create(name, sched)
            if cpus:
                for p in self._cpus_arg(cpus):
                    self.pool_cpu_add(pid, p)
            return pid

    def pool_destroy(self, pool):
        with self.lock:
            p = self._pool(pool)
            for c in self.engine.pool_info(p)["cpus"]:
                self.engine.pool_unassign(p, c)
            self.engine.pool_destroy(p)
            return 0

    def pool_rename(self, pool, name: str):
        with self.lock:
            return self.engine.pool_rename(self._pool(pool), name)

    def pool_cpu_add(self, pool, cpu):
        with self.lock:
            p = self._pool(pool)
            for c in self._cpus_arg(cpu):
                owner = self.engine.partition_info(c)["pool"]
                if owner == p:
                    continue
                if owner >= 0:
                    raise RpcError(f"cpu {c} is in cpupool {owner}", -16)
                self.engine.pool_assign(p, c)
            return 0

    def pool_cpu_remove(self, pool, cpu):
        with self.lock:
            p = self._pool(pool)
            for c in self._cpus_arg(cpu):
                self.engine.pool_unassign(p, c)
            return 0

    def pool_migrate(self, domain, pool):
        with self.lock:
            return self.engine.tenant_move(self._resolve(domain), self._pool(pool))

    def pool_xgmi_split(self):
        """cpupool-numa-split analog: one pool per GPU ("Pool-gpu<N>");
        tenants of Pool-0 stay on the first GPU's pool."""
        with self.lock:
            made = []
            for g in self.gpus[1:]:
                name = f"Pool-gpu{g}"
                pid = self.engine.pool_create(name, self.engine.sched_name(0))
                for (gg, x, c), part in self.part_of.items():
                    if gg == g:
                        self.engine.pool_unassign(0, part)
                        self.engine.pool_assign(pid, part)
                made.append(pid)
            if self.gpus:
                self.engine.pool_rename(0, f"Pool-gpu{self.gpus[0]}")
            return made

    def pause(self, domain):
        return self.engine.pause(self._resolve(domain))

    def unpause(self, domain):
        return self.engine.unpause(self._resolve(domain))

    def slot_list(self, domains: Optional[List] = None):
        ts = [self._resolve(d) for d in domains] if domains else self.engine.tenants()
        out = []
        for t in ts:
            name = self.engine.tenant_info(t).name
            for i in range(self.engine.tenant_info(t).nslots):
                s = self.engine.slot_info(self.engine.slot_id(t, i))
                aff = self.lib  # affinity decoded below
                out.append({"name": name, "id": t, "slot": i, "cpu": s["processor"], "state": s["runstate"],
                            "running": bool(s["is_running"]), "time_s": s["run_ns"] / 1e9, "credit": s["credit"],
                            "pri": s["pri"]})
        return out

    def slot_pin(self, domain, slot, cpus):
        t = self._resolve(domain)
        parts = self._cpus_arg(cpus)
        n = self.engine.tenant_info(t).nslots
        idx = list(range(n)) if str(slot) == "all" else [int(slot)]
        for i in idx:
            self.engine.pin(t, i, parts)
        return 0

    def slot_set(self, domain, n: int):
        return self.engine.set_nslots(self._resolve(domain), int(n))

    def debug_keys(self, keys: str):
        return self.engine.debug_keys(keys)

    def dmesg(self, clear: bool = False):
        return self.engine.dmesg(clear)

    def trace(self, max_records: int = 4096, from_start: bool = False):
        return [[r.t_ns, r.event, r.cpu, list(r.a)] for r in self.engine.trace(max_records, from_start)]

    def perfc(self, reset: bool = False):
        pc = self.engine.perfc()
        if reset:
            self.engine.perfc_reset()
        return pc

    def perfc_prom(self):
        """perfc + lock profile in the Prometheus text format (scrape target)."""
        return self.engine.perfc_prometheus()

    def lockprof(self, reset: bool = False):
        """xenlockprof analog: the engine mutex's lock/block counts and times."""
        return self.engine.lockprof(reset=bool(reset))

    def watchdog(self, domain, id: int = 0, timeout_ms: int = 0):
        """SCHEDOP_watchdog on behalf of a tenant (the shim's watchdog())."""
        return self.engine.watchdog(self._resolve(domain), int(id), int(timeout_ms))

    def mon(self, reset: bool = False):
        """xenmon analog (X:tools/xenmon/README): per-tenant share of the
        interval since the previous call that its slots spent running
        ("gotten"), runnable but not running ("waited") and blocked, plus
        dispatches per second, summed over slots and normalised per slot."""
        now = self.engine.now()
        cur = {}
        for t in self.engine.tenants():
            i = self.engine.tenant_info(t)
            tot = {"run": 0, "runnable": 0, "blocked": 0, "execs": 0}
            for k in range(i.nslots):
                si = self.engine.slot_info(self.engine.slot_id(t, k))
                tot["run"] += si["run_ns"]
                tot["runnable"] += si["runnable_ns"]
                tot["blocked"] += si["blocked_ns"]
                tot["execs"] += si["sched_count"]
            cur[t] = (i.name, i.nslots, tot)
        prev_t, prev = getattr(self, "_mon_prev", (None, {}))
        self._mon_prev = (now, cur)
        if reset or prev_t is None or now <= prev_t:
            return {"interval_s": 0.0, "tenants": []}
        dt = now - prev_t
        rows = []
        for t, (name, n, tot) in cur.items():
            p = prev.get(t, (name, n, {k: 0 for k in tot}))[2]
            d = {k: tot[k] - p[k] for k in tot}
            span = dt * max(1, n)
            rows.append({"id": t, "name": name, "slots": n, "gotten_pct": 100.0 * d["run"] / span,
                         "waited_pct": 100.0 * d["runnable"] / span, "blocked_pct": 100.0 * d["blocked"] / span,
                         "execs_per_s": d["execs"] / (dt / 1e9)})
        return {"interval_s": dt / 1e9, "tenants": rows}

    def top(self):
        """xentop analog: per-tenant share, quantum, phase, miss rate, counters."""
        now = self.engine.now()
        rows = []
        for t in self.engine.tenants():
            i = self.engine.tenant_info(t)
            rows.append({"id": t, "name": i.name, "pool": i.pool, "slots": i.nslots, "active": i.active_slots,
                         "run_s": i.run_ns / 1e9, "tslice_us": i.tslice_us, "phase": i.phase,
                         "miss_rate": i.cache_miss_rate, "cpi": i.cpi, "pmc": dict(zip(PMC_NAMES, i.pmc)),
                         "reports": i.report_count, "weight": i.weight, "cap": i.cap,
                         "class": self.engine.lib.gpbs_tenant_class(self.engine.h, t),
                         "vpmu": self.engine.tenant_vpmu(t)})
        parts = [self.engine.partition_info(p) for p in range(self.engine.num_partitions)]
        return {"now_ns": now, "tenants": rows, "partitions": parts}

    def register(self, name: str, slots: int = 8, weight: int = -1, cap: int = -1, pool=None, pid: int = 0):
        """A tenant process attaches: creates (or reuses) its tenant and binds a
        control page.  Returns what the shim needs to open the region."""
        with self.lock:
            try:
                t = self.engine.tenant_find(name)
            except Exception:
                t = self.create(name=name, slots=slots, weight=weight, cap=cap, pool=pool)
            if t in self.pages:
                page = self.pages[t]
            else:
                used = set(self.pages.values())
                page = next(i for i in range(self.lib.gpbs_ctl_ntenants(self.ctl)) if i not in used)
                self.pages[t] = page
                self.lib.gpbs_ctl_assign(self.ctl, page, t)
            self.engine.heartbeat(t)
            if pid:
                self.pids[t] = int(pid)
            return {"tenant": t, "page": page, "ctl": self.ctl_name, "nctx": self.nctx, "se_mode": self.se_mode,
                    "partitions": {f"{g}:{x}:{c}": p for (g, x, c), p in self.part_of.items()}}

    def unregister(self, name: str, destroy: bool = True):
        with self.lock:
            t = self.engine.tenant_find(name)
            self.engine.block(t)
            if destroy:
                return self.destroy(t)
            return 0

    def snapshot(self, path: Optional[str] = None):
        path = path or self.state_path
        if not path:
            raise RpcError("no state path", -22)
        snap.save(self.engine, path, extra={"pages": {str(k): v for k, v in self.pages.items()}})
        return path

    def restore(self, path: str):
        with self.lock:
            doc = snap.restore(self.engine, path)
            return {"tenants": len(doc.get("tenants", []))}

    def advance_us(self, us: float):
        """Simulated clock only: advance time (tests, replay)."""
        if not self.sim:
            raise RpcError("advance_us requires --sim", -22)
        self.engine.advance(self.engine.now() + int(us * 1000))
        return self.engine.now()

    def _handlers(self):
        names = ["info", "create", "destroy", "domain_list", "domain_sched_get", "domain_sched_set",
                 "domain_sched_ext_get", "domain_sched_ext_set", "arinc653_get", "arinc653_set",
                 "pool_params_get", "pool_params_set", "pool_list", "pool_create", "pool_destroy", "pool_rename",
                 "pool_cpu_add", "pool_cpu_remove", "pool_migrate", "pool_xgmi_split", "pause", "unpause",
                 "slot_list", "slot_pin", "slot_set", "debug_keys", "dmesg", "trace", "perfc", "top", "register",
                 "unregister", "snapshot", "restore", "advance_us", "perfc_prom", "lockprof", "watchdog", "mon"]
        return {n: getattr(self, n) for n in names}

    # ------------------------------------------------------------ reaper
    @staticmethod
    def _alive(pid: int) -> bool:
        try:
            os.kill(pid, 0)
        except ProcessLookupError:
            return False
        except PermissionError:
            return True
        try:  # a zombie child counts as dead
            with open(f"/proc/{pid}/stat") as f:
                return f.read().rsplit(")", 1)[1].split()[0] != "Z"
        except OSError:
            return False

    def reap(self) -> List[str]:
        """Failure detection (S13): destroy tenants whose registered process
        is gone, freeing their partitions and control page.  Tenants that
        merely stop heartbeating are paused by the engine (heartbeat_check)
        and resume nothing until they re-register."""
        dead = []
        with self.lock:
            for t, pid in list(self.pids.items()):
                if not self._alive(pid):
                    name = self.engine.tenant_info(t).name
                    try:
                        self.destroy(t)
                    except Exception:
                        self.pids.pop(t, None)
                    dead.append(name)
                    self.reaped.append(name)
        return dead

    def _reaper(self, period: float):
        while not self._stop_ev.wait(period):
            try:
                self.reap()
            except Exception as e:  # pragma: no cover
                print(f"[gpbsd] reaper: {e}", file=sys.stderr)

    # ---------------------------------------------------------------- run
    def start(self, reaper_s: float = 0.2):
        self.server.start()
        if not self.sim:
            self.engine.start()
        self.running = True
        self._stop_ev = threading.Event()
        self._reaper_th = None
        if reaper_s > 0:
            self._reaper_th = threading.Thread(target=self._reaper, args=(reaper_s,), daemon=True,
                                               name="gpbsd-reaper")
            self._reaper_th.start()
        return self

    def stop(self):
        """Orderly teardown: the reaper is joined before anything it touches
        goes away, RPC handlers are stopped, and the control-page bridge is
        closed BEFORE the GPU context (ctl_close reinstalls the actuator ops
        it chained at bind time; they must not point at a freed GpuCtx)."""
        if self.state_path:
            try:
                self.snapshot(self.state_path)
            except Exception as e:  # pragma: no cover
                print(f"[gpbsd] snapshot failed: {e}", file=sys.stderr)
        self.running = False
        ev = getattr(self, "_stop_ev", None)
        if ev is not None:
            ev.set()
        th = getattr(self, "_reaper_th", None)
        if th is not None:
            th.join()
            self._reaper_th = None
        self.server.stop()
        with self.lock:
            if not self.sim:
                self.engine.stop()
            self.lib.gpbs_ctl_close(self.ctl, 1)
            if self.gpu_ctxs:
                self.engine.mux_clear()
                for g in self.gpu_ctxs:
                    close = getattr(g, "close", None)
                    if close:
                        close()
                self.gpu_ctxs = []
                self.gpu_ctx = None
            self.engine.close()


def cfgmod_min_tslice() -> int:
    # Q1: the new API accepts the reference boot default (100us); xl's own
    # floor (1000us) is available via GPBS_XL_STRICT=1.
    return 1000 if os.environ.get("GPBS_XL_STRICT") == "1" else 100


def main(argv=None):
    ap = argparse.ArgumentParser(prog="gpbsd")
    ap.add_argument("--socket", default=DEFAULT_SOCKET)
    ap.add_argument("--gpus", default="0", help="comma list of GPU indices managed by this daemon")
    ap.add_argument("--nctx", type=int, default=2)
    ap.add_argument("--sim", action="store_true", help="simulated clock (no GPU, tests)")
    ap.add_argument("--profile", default="mi355x", choices=["mi355x", "reference"])
    ap.add_argument("--config", default=None)
    ap.add_argument("--state", default=None, help="snapshot file (restored at start, written on SIGTERM)")
    ap.add_argument("--snapshot-s", type=float, default=0.0)
    ap.add_argument("--attach-gpu", action="store_true", help="drive the partition table of --gpus[0] in-process")
    a = ap.parse_args(argv)
    d = Daemon(a.socket, gpus=[int(x) for x in a.gpus.split(",") if x != ""], nctx=a.nctx, sim=a.sim,
               profile=a.profile, config_path=a.config, state_path=a.state, attach_gpu=a.attach_gpu)
    d.start()
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    print(f"[gpbsd] serving {a.socket} ({d.engine.num_partitions} partitions)", flush=True)
    last = time.monotonic()
    while not stop.wait(0.2):
        if a.snapshot_s and a.state and time.monotonic() - last > a.snapshot_s:
            d.snapshot(a.state)
            last = time.monotonic()
    d.stop()


if __name__ == "__main__":
    main()
