"""GPU clock / power / throttle record (pbs_amd/utils/gpustate.py): the
window summary over a fake SMU source, and graceful absence on a CPU box."""
import time

from pbs_amd.utils import gpustate as G


class FakeSrc:
    def __init__(self):
        self.k = 0

    def read(self):
        self.k += 1
        # 10 ticks of accumulation per read, 4 of them in PPT (power) throttling
        return {"gfxclk_mhz": 2000.0 + self.k, "uclk_mhz": 2000.0, "power_w": 1300.0 + 10 * self.k,
                "temp_hotspot_c": 50.0 + self.k, "acc": 10.0 * self.k, "ppt_acc": 4.0 * self.k,
                "thm_acc": 0.0, "energy_acc": 100.0 * self.k}

    def close(self):
        pass


def test_window_summary_from_fake_source():
    r = G.GpuStateRecorder(source=FakeSrc(), period_s=0.01).start()
    t0 = r.now()
    time.sleep(0.2)
    t1 = r.now()
    r.stop()
    w = r.window(t0, t1)
    assert w["n"] >= 5
    assert 2000 < w["gfxclk_mhz"] < 2100 and w["power_w"] > 1300
    assert w["temp_hotspot_c_max"] > 50
    assert abs(w["ppt_frac"] - 0.4) < 1e-9 and w["thm_frac"] == 0.0
    assert w["energy_acc_delta"] > 0
    assert r.window(t1 + 10, t1 + 20) == {"source": r.source, "n": 0}


def test_not_supported_markers_are_dropped():
    assert G._num("N/A") is None and G._num(0xFFFF) is None and G._num(0xFFFFFFFF) is None
    assert G._num(1234) == 1234.0
    assert G._mean_valid([2000, 0xFFFF, 2100, 0]) == 2050.0


def test_no_gpu_box_yields_no_source():
    r = G.GpuStateRecorder(bdf="ffff:ff:1f.7")
    # a BDF that exists nowhere: no amdsmi handle, no sysfs device
    assert r.src is None or r.source is not None
    r.start()
    r.stop()
