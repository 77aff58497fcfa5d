"""bench.py contract under torchrun on CPU/gloo (2 ranks): one JSON line from rank 0 with the driver's keys."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


@pytest.mark.parametrize("method", ["zero", "ddp", "fsdp", "tp"])
def test_bench_torchrun_gloo_two_ranks(method, free_port):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--backend", "gloo", "--method", method,
           "--model_size", "64", "--layers", "2", "--batch_size", "2", "--seq_len", "16", "--dtype", "fp32"]
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert KEYS <= set(rec) and rec["value"] > 0 and rec["finite"]
    assert rec["config"]["global_batch"] == (2 if method == "tp" else 4)
