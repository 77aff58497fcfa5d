"""Compute-queue reservation (utils/streams.py, csrc/elementwise.hip dllm_queue_reserve / dllm_queue_shared).

Run in a fresh interpreter (the reservation must precede torch's stream pool): after ``reserve_compute_queue`` no
torch pool stream -- the engine's side streams and ProcessGroupNCCL's collective streams come from that pool -- runs on
the compute (null) stream's hardware queue, at HIP's default of 4 queues per process.  The probe itself is checked on
a stream pair that must share a queue (the null stream with itself through a second handle is not expressible, so a
blocker found by the reservation is used)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import json, torch
import dllm
from dllm.utils import streams
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
n = streams.reserve_compute_queue(0)
side = {f"s{i}": torch.cuda.Stream() for i in range(8)}
for st in side.values():
    with torch.cuda.stream(st):
        torch.zeros(1, device="cuda").add_(1)
torch.cuda.synchronize()
rep = streams.queue_report(0, side)
print("JSON" + json.dumps({"blockers": n, "report": rep}))
"""


@pytest.mark.parametrize("queues", ["4", "8"])
def test_reserved_compute_queue_is_exclusive(queues):
    env = dict(os.environ, PYTHONPATH=ROOT, GPU_MAX_HW_QUEUES=queues)
    r = subprocess.run([sys.executable, "-c", SCRIPT], capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("JSON")][0][4:])
    assert out["blockers"] >= 1, out          # some candidates landed on the compute queue and were kept
    rep = out["report"]
    assert rep["compute_queue_exclusive"], rep
    assert rep["side_streams_on_compute_queue"] == [] and rep["pool_streams_on_compute_queue"] == 0


def test_probe_detects_sharing_without_reservation():
    """Without the reservation, HIP's placement puts some of torch's 32 pool streams on the compute queue at 4 queues
    (the collision the reservation prevents) -- and the probe sees it."""
    script = SCRIPT.replace("n = streams.reserve_compute_queue(0)", "n = 0")
    env = dict(os.environ, PYTHONPATH=ROOT, GPU_MAX_HW_QUEUES="4")
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rep = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("JSON")][0][4:])["report"]
    assert rep["pool_streams_on_compute_queue"] > 0, rep
