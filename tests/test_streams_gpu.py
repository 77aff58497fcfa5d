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


ROLE_SCRIPT = r"""
import json, os, sys, time, ctypes, torch
import torch.distributed as dist
import dllm
from dllm import _native
from dllm.utils import streams
from dllm.parallel.mesh import Mesh, init_distributed
backend = sys.argv[1]
os.environ["LOCAL_RANK"] = "0"
init_distributed("nccl", 0, 1, "127.0.0.1", 29000 + os.getpid() % 1000)   # reserves the compute queue first
dev = torch.device("cuda", 0)
mesh = Mesh.build(1, 1, force=True, comm_backend=backend, device=dev)
rs = dict(mesh.role_streams)
rep = streams.role_queue_report(dev, rs)
out = {"role_streams": {k: (v is not None) for k, v in rs.items()}, "report": rep}
if backend == "torch":
    # the identified stream IS the process group's: a collective issued on dp_ag queues behind a spin on that stream,
    # and not behind a spin on dp_rs's stream (a different queue)
    sink = torch.zeros(1024, device=dev)
    def delay(spin_stream):
        torch.cuda.synchronize()
        rc = _native.lib().dllm_occupy(1, 64, ctypes.c_float(60000.0), ctypes.c_void_p(sink.data_ptr()),
                                       ctypes.c_void_p(spin_stream))
        assert rc == 0, rc
        t = torch.ones(256, device=dev)
        t0 = time.perf_counter()
        w = dist.all_reduce(t, group=mesh.groups["dp_ag"], async_op=True)
        while not w.is_completed():
            time.sleep(0.0005)
        dt = time.perf_counter() - t0
        torch.cuda.synchronize()
        return dt * 1e3
    out["delay_own_ms"] = delay(rs["dp_ag"])
    out["delay_other_ms"] = delay(rs["dp_rs"])
mesh.destroy()
print("JSON" + json.dumps(out))
dist.destroy_process_group()
"""


@pytest.mark.parametrize("backend", ["torch", "native"])
def test_role_communicators_on_distinct_queues(backend):
    """the FSDP gather (dp_ag) and reduce-scatter (dp_rs) communicators' streams run on different
    hardware queues, and no role communicator shares the compute stream's -- measured on the real process-group streams
    (torch: identified in torch's stream pool and steered at mesh build; native: our own streams), at HIP's default 4
    queues.  For torch the identification is checked behaviourally: a dp_ag collective waits for a 60 ms spin on the
    identified stream but not for one on dp_rs's."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("GPU_MAX_HW_QUEUES", None)
    r = subprocess.run([sys.executable, "-c", ROLE_SCRIPT, backend], capture_output=True, text=True, timeout=300,
                       cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("JSON")][0][4:])
    assert all(out["role_streams"].values()), out
    assert out["report"]["role_queue_conflicts"] == [], out
    assert ["dp_ag", "dp_rs"] not in out["report"]["queue_sharing_pairs"], out
    if backend == "torch":
        assert out["delay_own_ms"] > 40.0, out
        assert out["delay_other_ms"] < 30.0, out


ENGINE_SCRIPT = r"""
import json, torch
import dllm
from dllm.models.ffn import init_ffn_params_device
from dllm.parallel.engine import FFNTrainer
from dllm.parallel.mesh import Mesh
from dllm.utils import streams
from dllm.utils.config import ModelConfig, TrainConfig
from dllm.utils.data import DeviceMockData
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
m = ModelConfig(model_size=4096, ffn_dim=16384, layers=1, act="relu")     # flagship layer: weight-gradient stream on
cfg = TrainConfig(model=m, batch_size=1, seq_len=1024, dtype="bf16", grad_dtype="fp32", optimizer="sgd",
                  wgrad_stream=True, wgrad_layout="tn")   # the TN layout keeps the weight-gradient side stream
eng = FFNTrainer(cfg, Mesh(), dev)          # no bench.py, no launcher: the engine reserves the queue itself
eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 1, dev))
data = DeviceMockData(cfg.tokens, m.D, torch.bfloat16, dev)
for i in range(3):
    x, dy = data.fill(i)
    eng.train_step(x, dy)
torch.cuda.synchronize()
side = {"wgrad": eng.wg_stream, "opt": getattr(eng, "opt_stream", None), "data": getattr(data, "_stream", None)}
side = {k: v for k, v in side.items() if v is not None}
print("JSON" + json.dumps({"sides": sorted(side), "report": streams.queue_report(0, side)}))
"""


def test_single_rank_engine_reserves_compute_queue():
    """a world==1 run that goes through neither bench.py nor the launcher (the Python API, train_ffns at
    N=1) still gets the compute-queue reservation -- FFNTrainer makes it before creating any side stream -- so at
    HIP's default 4 queues no side stream and no pool stream shares the compute stream's queue."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("GPU_MAX_HW_QUEUES", None)
    r = subprocess.run([sys.executable, "-c", ENGINE_SCRIPT], capture_output=True, text=True, timeout=300, cwd=ROOT,
                       env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("JSON")][0][4:])
    assert "wgrad" in out["sides"], out
    rep = out["report"]
    assert rep["compute_queue_exclusive"], rep
    assert rep["side_streams_on_compute_queue"] == [] and rep["pool_streams_on_compute_queue"] == 0, rep
