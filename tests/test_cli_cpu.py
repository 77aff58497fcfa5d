"""The reference-compatible CLI (train_ffns.py:342-391) on CPU/gloo."""
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cli(*args, port):
    return subprocess.run([sys.executable, os.path.join(ROOT, "train_ffns.py"), *args, "--master_port", str(port)],
                          capture_output=True, text=True, timeout=600, cwd=ROOT)


def test_method0_all_methods_agree(free_port):
    r = _cli("-s", "4", "-bs", "2", "-n", "8", "-l", "2", "-d", "16", "-m", "0", "-r", "3", "--lr", "0.01",
             "--strict", port=free_port)
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout
    assert "ARGS:" in out and "PARAMS: 4_096" in out
    for fn in ("train_1gpu", "train_ddp", "train_fsdp", "train_tp"):
        assert f"{fn} takes" in out
    assert "SoftAssertionError" not in out


def test_hybrid_method_and_extended_flags(free_port):
    r = _cli("-s", "2", "-bs", "1", "-n", "8", "-l", "2", "-d", "16", "-m", "5", "-r", "3", "--nprocs", "4",
             "--tp", "2", "--act", "silu", "--gated", "--ffn_dim", "32", "--optimizer", "adam", port=free_port)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "train_hybrid takes" in r.stdout
