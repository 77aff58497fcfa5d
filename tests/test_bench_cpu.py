"""bench.py contract under torchrun on CPU/gloo (2 ranks): one JSON line from rank 0 with the driver's keys."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _run(free_port, *extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--backend", "gloo",
           "--model_size", "64", "--layers", "2", "--batch_size", "2", "--seq_len", "16", "--dtype", "fp32",
           "--mp_ffn_dim", "128", "--llama_ffn_dim", "128", "--llama_layers", "2", *extra]
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert KEYS <= set(rec) and rec["value"] > 0 and rec["finite"]
    return rec


@pytest.mark.parametrize("method", ["ddp", "fsdp", "tp"])
def test_bench_torchrun_gloo_two_ranks(method, free_port):
    rec = _run(free_port, "--method", method, "--methods", "none")
    assert rec["config"]["global_batch"] == (2 if method == "tp" else 4)
    assert "methods" not in rec
    if method == "tp":
        assert "F128" in rec["config"]["model"] and rec["scaling"] == "strong"  # the MP config's FFN width


def test_bench_methods_side_by_side(free_port):
    """The default run: ZeRO-2 headline plus ddp / zero / fsdp / tp / hybrid timed side by side on their own engines
    (the reference's --method 0, train_ffns.py:373-384; hybrid = BASELINE config 5, FSDP x TP on a SwiGLU stack)."""
    rec = _run(free_port)
    assert rec["config"]["parallelism"] == "dp2-zero2" and rec["config"]["global_batch"] == 4
    assert set(rec["methods"]) == {"ddp", "zero", "fsdp", "tp", "hybrid"}   # fsdp_copy: N = 1 only
    for name, m in rec["methods"].items():
        assert m["value"] > 0 and m["ms_per_step"] > 0 and m["finite"], name
        assert {"peak_hbm_gib", "parallelism", "model", "state_gib"} <= set(m), name
        # steady-state windows: >= 150 ms of warm-up and ~300 ms timed (or the step cap); the timed window is sized
        # from the warm step time, which reads noisy on shared CPU cores (the GPU runs check >= 300 ms)
        assert m["warmup_ms"] >= 150 and (m["timed_ms"] >= 200 or m["steps"] >= 1000), (name, m)
    assert rec["methods"]["tp"]["parallelism"] == "tp2" and "L1 D64 F128" in rec["methods"]["tp"]["model"]
    assert rec["methods"]["fsdp"]["parallelism"] == "fsdp2"
    assert rec["methods"]["hybrid"]["parallelism"] == "fsdp1xtp2" and "L2 D64 F128 swiglu-silu" in rec["methods"]["hybrid"]["model"]


def test_bench_side_methods_deadline_keeps_headline(free_port):
    """A side-by-side method that overruns --side_deadline_s cannot cost the headline: rank 0 still prints the one
    line (methods finished so far plus the cut-off one as an error) and every rank exits 0."""
    rec = _run(free_port, "--side_deadline_s", "0.05")
    assert "cut off" in rec["note"]
    assert any("error" in m for m in rec["methods"].values())


def test_bench_self_launches_ranks():
    """``python bench.py --gpus 2`` with no launcher starts its own two ranks (the reference starts one worker per GPU
    from a plain ``python train_ffns.py``, train_ffns.py:184-191): one JSON line, world_size 2, every role
    communicator of the headline spanning both ranks."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--backend", "gloo", "--model_size", "64", "--layers", "2", "--batch_size", "2", "--seq_len", "16",
           "--dtype", "fp32", "--methods", "none"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2 and rec["launcher"] == "self"
    assert rec["config"]["parallelism"] == "dp2-zero2" and rec["config"]["global_batch"] == 4
    assert rec["comm_sizes"] and all(v == 2 for v in rec["comm_sizes"].values()), rec["comm_sizes"]


def test_bench_self_launch_propagates_rank_failure():
    """A rank that dies fails the whole self-launched run (non-zero exit), instead of hanging or printing a line."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--backend", "gloo", "--model_size", "64", "--layers", "2", "--batch_size", "2", "--seq_len", "16",
           "--dtype", "fp32", "--methods", "none", "--no_such_flag"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_self_launch_four_ranks_all_methods():
    """The driver's plain ``python bench.py --gpus 4`` shape: four self-launched ranks, every side method on its own
    mesh (hybrid = FSDP 2 x TP 2), communicator sizes reported per method, the differential exposed-comm field present."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1", "--warmup", "1",
           "--backend", "gloo", "--model_size", "64", "--layers", "2", "--batch_size", "2", "--seq_len", "16",
           "--dtype", "fp32", "--mp_ffn_dim", "128", "--llama_ffn_dim", "128", "--llama_layers", "2",
           "--method_steps", "1", "--diff_pairs", "1", "--diff_steps", "1", "--observe_steps", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert rec["world_size"] == 4 and rec["config"]["parallelism"] == "dp4-zero2"
    m = rec["methods"]
    assert m["hybrid"]["parallelism"] == "fsdp2xtp2" and m["hybrid"]["comm_sizes"]["tp"] == 2
    assert m["hybrid"]["comm_sizes"]["dp_rs"] == 2 and m["tp"]["comm_sizes"] == {"tp": 4}
    assert all("exposed_ms_diff" in m[k]["comm"] for k in ("ddp", "zero", "fsdp", "hybrid"))


def test_bench_self_launch_eight_ranks_all_methods():
    """The driver's largest shape, ``python bench.py --gpus 8`` with no launcher, rehearsed over gloo on the CPU: eight
    self-launched ranks, headline ZeRO-2 over 8, MP over 8, hybrid FSDP 4 x TP 2, every role communicator sized as
    RCCL would see it."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup", "1",
           "--backend", "gloo", "--model_size", "64", "--layers", "2", "--batch_size", "1", "--seq_len", "16",
           "--dtype", "fp32", "--mp_ffn_dim", "256", "--llama_ffn_dim", "128", "--llama_layers", "2",
           "--method_steps", "1", "--diff_pairs", "1", "--diff_steps", "1", "--observe_steps", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=1200, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1   # rank 0 alone prints
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8 and rec["world_size"] == 8 and rec["launcher"] == "self"
    assert rec["config"]["parallelism"] == "dp8-zero2" and rec["comm_sizes"]["dp_rs"] == 8
    m = rec["methods"]
    assert m["tp"]["comm_sizes"] == {"tp": 8}
    assert m["hybrid"]["parallelism"] == "fsdp4xtp2" and m["hybrid"]["comm_sizes"]["dp_ag"] == 4
    assert all(m[k]["finite"] for k in m)


def test_bench_data_note_reports_non_finite():
    """The JSON ``data`` string is derived from the run's ``finite`` flag: a run whose weights
    overflowed (e.g. ``--init_scale 0.02`` on the flagship stack) must say NON-FINITE, never "finite data throughout"."""
    sys.path.insert(0, ROOT)
    import bench

    bad = bench.data_note(0.02, False)
    assert "NON-FINITE" in bad and "finite data throughout" not in bad
    good = bench.data_note("fan_in", True, overlap=True)
    assert "finite data throughout" in good and "NON-FINITE" not in good and "side stream" in good


def test_bench_zero_copy_entry_single_rank(free_port):
    """At N = 1 the side-by-side methods include zero_copy: ZeRO-2 over size-1 communicators whose reduce-scatters and
    all-gathers copy (separate shard, all-gather sink), at two GEMM blocks per CU -- the N>1 headline's schedule."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "1", "--warmup", "1",
           "--backend", "gloo", "--model_size", "64", "--layers", "2", "--batch_size", "2", "--seq_len", "16",
           "--dtype", "fp32", "--methods", "zero", "--method_steps", "1", "--diff_pairs", "0", "--observe_steps", "0",
           "--side_warmup_ms", "1", "--side_timed_ms", "1"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PYTHONPATH=ROOT, MASTER_PORT=str(free_port))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert set(rec["methods"]) == {"zero", "zero_copy"}
    assert rec["methods"]["zero_copy"]["parallelism"] == "dp1-zero2-forcecomm" and rec["methods"]["zero_copy"]["finite"]
