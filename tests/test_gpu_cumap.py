"""The CU-mask bit layout every SE-exclusive policy assumes holds on this GPU
(scripts/cu_map_check.py, in a child process so its four queues do not stay
in the test process): a queue masked to shader engine s of every XCD runs
its workgroups on SE s only, on all 8 XCDs."""
import json
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cu_mask_bits_map_to_shader_engines():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "cu_map_check.py")], capture_output=True,
                       text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    print(json.dumps(res))
    for s, r in res["se"].items():
        assert r["workgroups"] > 0 and r["xcds"] == list(range(8)), (s, r)
        assert set(r["real_se"]) == {s}, (s, r)
    assert res["ok"]
