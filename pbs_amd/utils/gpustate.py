"""GPU clock / power / temperature / throttle record, per run.

The live-counter drift of round 3 (the GPU ran ~11 % slower after many
device-counting samples, VERDICT r3 missing #1) could be a DVFS / power
state or a queue-to-pipe effect.  This module tells them apart by recording,
from a host thread, what the SMU reports while the GPU works: gfx clock
(average and current, per XCD), memory clock, socket power, hotspot / HBM
temperature, and the PPT (power) and thermal throttle residency counters.
It reads through amdsmi (``amdsmi_get_gpu_metrics_info``) when that works
for the current user and falls back to the amdgpu sysfs files
(``pp_dpm_sclk``, hwmon ``power1_average`` / ``temp*_input``) otherwise; a
box where neither is readable yields ``{"source": None}`` and the bench goes
on.  The reference's analogue is the perfctr TSC / clock bookkeeping that
makes its counter deltas comparable across samples
(X:xen/arch/x86/perfctr.c:1547-1572).

    rec = GpuStateRecorder(bdf="0000:05:00.0", period_s=0.25)
    rec.start()
    t0 = rec.now(); ...work...; t1 = rec.now()
    rec.window(t0, t1)   # {"gfxclk_mhz": ..., "power_w": ..., "ppt_frac": ...}
    rec.stop()
"""
from __future__ import annotations

import glob
import os
import threading
import time
from typing import Dict, List, Optional

_NA = (None, "N/A")


def _num(v) -> Optional[float]:
    if v in _NA or isinstance(v, str):
        return None
    try:
        f = float(v)
    except (TypeError, ValueError):
        return None
    return None if f in (0xFFFF, 0xFFFFFFFF, float(0xFFFFFFFFFFFFFFFF)) else f  # "not supported" markers


def _mean_valid(xs) -> Optional[float]:
    if not isinstance(xs, (list, tuple)):
        return _num(xs)
    v = [_num(x) for x in xs]
    v = [x for x in v if x is not None and 0 < x < 0xFFFF]
    return sum(v) / len(v) if v else None


def device_bdf(device: int = 0) -> Optional[str]:
    """PCI address ("dddd:bb:dd.f") of torch device `device` (initialises
    the HIP runtime)."""
    try:
        import torch
        p = torch.cuda.get_device_properties(device)
        return "%04x:%02x:%02x.0" % (int(getattr(p, "pci_domain_id", 0)), int(p.pci_bus_id), int(p.pci_device_id))
    except Exception:
        return None


def bdf_key(bdf: Optional[str]):
    """(domain, bus, device) of a "dddd:bb:dd.f" / "bb:dd.f" address, the
    function dropped; None when it does not parse."""
    if not bdf:
        return None
    try:
        parts = bdf.lower().split(":")
        dom = int(parts[0], 16) if len(parts) == 3 else 0
        bus = int(parts[-2], 16)
        dev = int(parts[-1].split(".")[0], 16)
        return (dom, bus, dev)
    except (ValueError, IndexError):
        return None


def bdf_mismatch(a: Optional[str], b: Optional[str]) -> bool:
    """True only when both addresses are known and name different devices
    (an unknown address is no evidence of a mismatch)."""
    ka, kb = bdf_key(a), bdf_key(b)
    return ka is not None and kb is not None and ka != kb


class _AmdSmi:
    def __init__(self, bdf: Optional[str]):
        import amdsmi
        self.m = amdsmi
        amdsmi.amdsmi_init()
        hs = amdsmi.amdsmi_get_processor_handles()
        self.h = None
        if bdf:
            for h in hs:
                try:
                    if amdsmi.amdsmi_get_gpu_device_bdf(h).lower() == bdf.lower():
                        self.h = h
                        break
                except Exception:
                    continue
        if self.h is None:
            if len(hs) != 1:
                raise RuntimeError("amdsmi: no handle for %s" % bdf)
            self.h = hs[0]
        self.read()  # raises if this user cannot read the metrics table

    def read(self) -> Dict[str, Optional[float]]:
        m = self.m.amdsmi_get_gpu_metrics_info(self.h)
        return {
            "gfxclk_avg_mhz": _num(m.get("average_gfxclk_frequency")),
            "gfxclk_mhz": _mean_valid(m.get("current_gfxclks")) or _num(m.get("current_gfxclk")),
            "uclk_mhz": _num(m.get("current_uclk")),
            "power_w": _num(m.get("current_socket_power")) or _num(m.get("average_socket_power")),
            "temp_hotspot_c": _num(m.get("temperature_hotspot")),
            "temp_mem_c": _num(m.get("temperature_mem")),
            "energy_acc": _num(m.get("energy_accumulator")),
            "acc": _num(m.get("accumulation_counter")),
            "ppt_acc": _num(m.get("ppt_residency_acc")),
            "thm_acc": _num(m.get("socket_thm_residency_acc")),
            "hbm_thm_acc": _num(m.get("hbm_thm_residency_acc")),
            "gfx_busy": _num(m.get("average_gfx_activity")),
        }

    def close(self):
        try:
            self.m.amdsmi_shut_down()
        except Exception:
            pass


class _Sysfs:
    def __init__(self, bdf: Optional[str]):
        dev = None
        for d in glob.glob("/sys/class/drm/card*/device"):
            real = os.path.realpath(d)
            if bdf is None or os.path.basename(real).lower() == (bdf or "").lower():
                if os.path.exists(os.path.join(d, "pp_dpm_sclk")):
                    dev = d
                    break
        if dev is None:
            raise RuntimeError("sysfs: no amdgpu device for %s" % bdf)
        self.dev = dev
        hw = glob.glob(os.path.join(dev, "hwmon", "hwmon*"))
        self.hw = hw[0] if hw else None
        self.read()

    @staticmethod
    def _rd(p) -> Optional[str]:
        try:
            with open(p) as f:
                return f.read()
        except OSError:
            return None

    def _dpm(self, name) -> Optional[float]:
        s = self._rd(os.path.join(self.dev, name))
        if not s:
            return None
        for line in s.splitlines():
            if line.rstrip().endswith("*"):
                for tok in line.split():
                    if tok.lower().endswith("mhz"):
                        return _num(tok[:-3])
        return None

    def read(self) -> Dict[str, Optional[float]]:
        out = {"gfxclk_mhz": self._dpm("pp_dpm_sclk"), "uclk_mhz": self._dpm("pp_dpm_mclk")}
        if self.hw:
            p = self._rd(os.path.join(self.hw, "power1_average")) or self._rd(os.path.join(self.hw, "power1_input"))
            out["power_w"] = float(p) / 1e6 if p else None
            t = self._rd(os.path.join(self.hw, "temp2_input")) or self._rd(os.path.join(self.hw, "temp1_input"))
            out["temp_hotspot_c"] = float(t) / 1e3 if t else None
        if all(v is None for v in out.values()):
            raise RuntimeError("sysfs: nothing readable")
        return out

    def close(self):
        pass


def open_source(bdf: Optional[str]):
    """The first readable metrics source for the GPU at `bdf`, or None."""
    for cls in (_AmdSmi, _Sysfs):
        try:
            return cls(bdf)
        except Exception:
            continue
    return None


class GpuStateRecorder:
    """Background sampler of the GPU's SMU state (clock, power, temperature,
    throttle residency) every `period_s`; `window(t0, t1)` summarises it."""

    def __init__(self, bdf: Optional[str] = None, period_s: float = 0.25, source=None):
        self.bdf = bdf
        self.period_s = period_s
        self.src = source if source is not None else open_source(bdf)
        self.samples: List[tuple] = []  # (t, dict)
        self._stop = threading.Event()
        self._th: Optional[threading.Thread] = None
        self._mu = threading.Lock()

    @property
    def source(self) -> Optional[str]:
        if self.src is None:
            return None
        return "amdsmi" if isinstance(self.src, _AmdSmi) else type(self.src).__name__.strip("_").lower()

    def now(self) -> float:
        return time.monotonic()

    def _one(self):
        try:
            d = self.src.read()
        except Exception:
            return
        with self._mu:
            self.samples.append((time.monotonic(), d))

    def _loop(self):
        while not self._stop.wait(self.period_s):
            self._one()

    def start(self) -> "GpuStateRecorder":
        if self.src is not None and self._th is None:
            self._one()
            self._th = threading.Thread(target=self._loop, name="gpbs-gpustate", daemon=True)
            self._th.start()
        return self

    def stop(self):
        self._stop.set()
        if self._th is not None:
            self._th.join(timeout=2.0)
            self._th = None
        if self.src is not None:
            self.src.close()

    def window(self, t0: float, t1: float) -> Dict[str, Optional[float]]:
        """Means over the samples in [t0, t1]; residency counters as the
        fraction of the window's accumulation ticks spent throttled."""
        with self._mu:
            win = [d for (t, d) in self.samples if t0 <= t <= t1]
        out: Dict[str, Optional[float]] = {"source": self.source, "n": len(win)}
        if not win:
            return out
        for k in ("gfxclk_mhz", "gfxclk_avg_mhz", "uclk_mhz", "power_w", "gfx_busy"):
            v = [d[k] for d in win if d.get(k) is not None]
            out[k] = round(sum(v) / len(v), 1) if v else None
        for k in ("temp_hotspot_c", "temp_mem_c"):
            v = [d[k] for d in win if d.get(k) is not None]
            out[k + "_max"] = max(v) if v else None
        a, b = win[0], win[-1]
        if a.get("acc") is not None and b.get("acc") is not None and b["acc"] > a["acc"]:
            dacc = b["acc"] - a["acc"]
            for k, name in (("ppt_acc", "ppt_frac"), ("thm_acc", "thm_frac"), ("hbm_thm_acc", "hbm_thm_frac")):
                if a.get(k) is not None and b.get(k) is not None:
                    out[name] = round((b[k] - a[k]) / dacc, 4)
        if a.get("energy_acc") is not None and b.get("energy_acc") is not None:
            out["energy_acc_delta"] = b["energy_acc"] - a["energy_acc"]
        return out
