"""RCCL code paths on one GPU: size-1 communicators run real collectives, streams and events.

Covers the native C++ RCCL layer (csrc/comm.cpp) and torch ProcessGroupNCCL role groups, and every
data-parallel engine path (DDP all-reduce, ZeRO-2 reduce-scatter/all-gather, FSDP gather ring + async
reduce-scatter) forced onto them, against the single-device (fused-optimizer) engine.
"""
import os

import pytest
import torch
import torch.distributed as dist

from dllm.models.ffn import init_ffn_layer
from dllm.parallel import selftest
from dllm.parallel.engine import FFNTrainer
from dllm.parallel.mesh import Mesh, init_distributed
from dllm.utils.config import ModelConfig, TrainConfig
from dllm.utils.data import reference_mock_data

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    os.environ["LOCAL_RANK"] = "0"
    init_distributed("nccl", 0, 1, "127.0.0.1", 29000 + os.getpid() % 1000)
    yield
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("backend", ["torch", "native"])
def test_role_collectives(pg, backend):
    dev = torch.device("cuda", 0)
    mesh = Mesh.build(1, 1, force=True, comm_backend=backend, device=dev)
    assert set(mesh.groups) == {"dp_ar", "dp_ag", "dp_rs", "tp"}
    selftest.check_collectives(mesh, dev)
    selftest.check_async_side_stream(1, dev)
    mesh.destroy()


def test_native_work_orders_streams(pg):
    """A collective on the role stream must see compute queued before it, and compute queued after
    wait() must see its result (event edges both ways)."""
    from dllm.parallel.rccl import NativeGroup

    dev = torch.device("cuda", 0)
    g = NativeGroup([0], "order", dev)
    x = torch.zeros(1 << 22, device=dev)
    for i in range(5):
        x.add_(1.0)                 # compute stream
        w = g.all_reduce(x)         # role stream waits on the compute event
        w.wait()                    # compute waits on the collective
        x.mul_(2.0)
    torch.cuda.synchronize()
    want = 0.0
    for _ in range(5):
        want = (want + 1.0) * 2.0
    assert torch.all(x == want)
    g.destroy()


def test_native_abort_error_path(pg):
    """ncclCommAbort path: a communicator with completed work aborts cleanly, and a mesh
    torn down with abort=True leaves no communicator behind."""
    from dllm.parallel.rccl import NativeGroup

    dev = torch.device("cuda", 0)
    g = NativeGroup([0], "abort", dev)
    x = torch.ones(1024, device=dev)
    g.all_reduce(x).wait()
    torch.cuda.synchronize()
    g.check_async_error()
    g.abort()
    assert g.comm is None
    g.destroy()  # idempotent after abort (releases the stream)
    mesh = Mesh.build(1, 1, force=True, comm_backend="native", device=dev)
    mesh.destroy(abort=True)
    assert not mesh.groups


def _run(dp_mode, backend, dtype="fp32", opt="sgd", force=True, fsdp_alias=True, zero_alias=True):
    D, F, L, T = 256, 1024, 2, 512
    gen = torch.Generator().manual_seed(9)
    layers = [init_ffn_layer(D, F, gen) for _ in range(L)]
    batches = list(reference_mock_data(torch.randint(100_000, (3,), generator=gen), T, D))
    cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=1, seq_len=T, dtype=dtype, grad_dtype="fp32",
                      lr=1e-2 if opt == "sgd" else 1e-3, optimizer=opt, dp_mode=dp_mode, force_comm=force,
                      comm_backend=backend, fsdp_alias=fsdp_alias, zero_alias=zero_alias)
    dev = torch.device("cuda", 0)
    mesh = Mesh.build(1, 1, force=force, comm_backend=backend, device=dev)
    eng = FFNTrainer(cfg, mesh, dev)
    eng.load_full_params(layers)
    cd = torch.bfloat16 if dtype == "bf16" else torch.float32
    for x, dy in batches:
        eng.train_step(x.to(dev, cd), dy.to(dev, cd))
    out = eng.gather_full_params()
    mesh.destroy()
    return out


@pytest.mark.parametrize("backend", ["torch", "native"])
@pytest.mark.parametrize("dp_mode", ["ddp", "zero", "fsdp"])
@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_dp_paths_match_single_device(pg, backend, dp_mode, opt):
    ref = _run("none", "torch", opt=opt, force=False)
    got = _run(dp_mode, backend, opt=opt)
    for g, w in zip(got, ref):
        for k in w:
            torch.testing.assert_close(g[k], w[k], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("backend", ["torch", "native"])
def test_fsdp_copying_rings_equal_aliased(pg, backend):
    """bench.py's fsdp_copy entry: FSDP at dp = 1 on its gather / gradient rings with real (copying) size-1 RCCL
    all-gathers and reduce-scatters gives bitwise the aliased schedule's parameters."""
    a = _run("fsdp", backend, dtype="bf16")
    b = _run("fsdp", backend, dtype="bf16", fsdp_alias=False)
    for g, w in zip(a, b):
        for k in w:
            assert torch.equal(g[k], w[k]), k


@pytest.mark.parametrize("backend", ["torch", "native"])
@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_zero_copying_collectives_equal_aliased(pg, backend, opt):
    """bench.py's zero_copy entry: ZeRO-2 at dp = 1 with a separate gradient shard and an all-gather sink (real copying
    size-1 RCCL reduce-scatters / all-gathers) gives bitwise the aliased schedule's parameters."""
    a = _run("zero", backend, dtype="bf16", opt=opt)
    b = _run("zero", backend, dtype="bf16", opt=opt, zero_alias=False)
    for g, w in zip(a, b):
        for k in w:
            assert torch.equal(g[k], w[k]), k


@pytest.mark.parametrize("backend", ["torch", "native"])
@pytest.mark.parametrize("dp_mode", ["ddp", "zero", "fsdp"])
def test_race_screen_serialized_equals_overlapped(pg, backend, dp_mode):
    """SURVEY §5.2 race screen on the GPU: serialized collectives + device syncs == overlapped, bitwise."""
    from dllm.parallel import comm

    a = _run(dp_mode, backend, dtype="bf16")
    comm.set_serialize(True)
    try:
        b = _run(dp_mode, backend, dtype="bf16")
    finally:
        comm.set_serialize(False)
    for g, w in zip(a, b):
        for k in w:
            assert torch.equal(g[k], w[k]), (dp_mode, k)


def test_native_single_process_rccl_selftest():
    """test_nccl.py analog: ncclCommInitAll over every visible device, group-fused AG/AR/RS of 128 fp32
    per rank against host expectations (csrc/tools/rccl_selftest.cpp)."""
    import os
    import subprocess

    import dllm
    from dllm import _build

    exe = os.path.join(_build.BIN, "dllm_rccl_selftest")
    if not os.path.exists(exe):
        _build.build_tools()
    env = dict(os.environ)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout
    for op in ("all_gather ok", "all_reduce ok", "reduce_scatter ok"):
        assert op in r.stdout


def test_elided_collective_keeps_dependency(pg):
    """exposed_ms_diff's reference steps: an elided collective returns at once but its wait() still orders the waiting
    stream after the issue point (the producer's kernels), like an infinitely fast collective."""
    from dllm.ops.elementwise import occupy_cus
    from dllm.parallel import comm

    dev = torch.device("cuda", 0)
    mesh = Mesh.build(1, 1, force=True, comm_backend="torch", device=dev)
    x = torch.zeros(1 << 20, device=dev)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    old = comm.set_elide(True)
    try:
        with torch.cuda.stream(side):
            occupy_cus(8, 3000.0, device=dev)   # 3 ms on the producer stream before the write
            x.fill_(1.0)
            w = comm.all_gather_into(x, x, mesh.group("dp_ag"), async_op=True)
        assert isinstance(w, comm.Elided)
        w.wait()
        y = x * 2.0
    finally:
        comm.set_elide(old)
    torch.cuda.synchronize()
    assert torch.all(y == 2.0)
    mesh.destroy()


@pytest.mark.parametrize("backend", ["torch", "native"])
def test_sync_all_reduce_on_current_stream_orders(pg, backend):
    """A synchronous all-reduce (async_op=False: on the caller's stream, no communicator-stream hop) sits between the
    compute stream's producer and consumer kernels."""
    from dllm.parallel import comm

    dev = torch.device("cuda", 0)
    mesh = Mesh.build(1, 1, force=True, comm_backend=backend, device=dev)
    x = torch.zeros(1 << 22, device=dev)
    for _ in range(5):
        x.add_(1.0)
        assert isinstance(comm.all_reduce(x, mesh.group("tp"), async_op=False), comm.Done)
        x.mul_(2.0)
    torch.cuda.synchronize()
    want = 0.0
    for _ in range(5):
        want = (want + 1.0) * 2.0
    assert torch.all(x == want)
    mesh.destroy()


def test_fsdp_side_stream_priority_bitwise(pg, monkeypatch):
    """The default side-stream policy puts the FSDP stream at high priority (utils/streams.py ``role``): only where
    the shard updates and step-boundary gathers are queued changes, so the result is bitwise the all-pool run's."""
    outs = []
    for mode in ("role", "pool"):
        monkeypatch.setenv("DLLM_SIDE_STREAMS", mode)
        D, F, L, T = 256, 1024, 3, 512
        gen = torch.Generator().manual_seed(21)
        layers = [init_ffn_layer(D, F, gen) for _ in range(L)]
        cfg = TrainConfig(model=ModelConfig(D, F, L), batch_size=1, seq_len=T, dtype="bf16", grad_dtype="bf16",
                          lr=1e-2, dp_mode="fsdp", force_comm=True, comm_backend="torch")
        dev = torch.device("cuda", 0)
        mesh = Mesh.build(1, 1, force=True, comm_backend="torch", device=dev)
        eng = FFNTrainer(cfg, mesh, dev)
        assert isinstance(eng.fsdp_stream, torch.cuda.ExternalStream) == (mode == "role")
        eng.load_full_params(layers)
        for x, dy in reference_mock_data(torch.tensor([5, 6, 7]), T, D):
            eng.train_step(x.to(dev, torch.bfloat16), dy.to(dev, torch.bfloat16))
        eng.fsdp_sync()
        torch.cuda.synchronize()
        outs.append(eng.master.clone())
        mesh.destroy()
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))


@pytest.mark.parametrize("gated", [False, True])
def test_tp_layers_w2_transposed_storage_bitwise(pg, gated):
    """Round 6: on row-major TP layers W2 is stored as W2ᵀ by default (``w2_storage='auto'``: the dgrad runs NT, fwd-2
    NN, dW2 through the TN kernels' transposed output map).  FSDP x TP over size-1 RCCL communicators (bench.py's
    hybrid entry at N=1), 2 steps: bitwise the row-major storage's parameters."""
    from dllm.models.ffn import init_ffn_params_device
    from dllm.utils.data import DeviceMockData

    dev = torch.device("cuda", 0)
    m = ModelConfig(model_size=2048, ffn_dim=8192, layers=2, act="silu" if gated else "relu", gated=gated)
    out = {}
    for storage in ("rowmajor", "auto"):
        cfg = TrainConfig(model=m, batch_size=1, seq_len=1024, dtype="bf16", grad_dtype="bf16", lr=1e-3,
                          optimizer="adam" if gated else "sgd", dp_mode="fsdp", force_comm=True, force_tp_comm=True,
                          w2_storage=storage)
        mesh = Mesh.build(1, 1, force=True, device=dev)
        eng = FFNTrainer(cfg, mesh, dev)
        assert eng.tp_comm and eng.fsdp and eng.w2t == (storage == "auto")
        eng.load_full_params(init_ffn_params_device(m.D, m.F, m.layers, 11, dev, gated=gated))
        data = DeviceMockData(cfg.tokens, m.D, torch.bfloat16, dev)
        ys = [eng.train_step(*data.fill(i)).clone() for i in range(2)]
        torch.cuda.synchronize()
        out[storage] = (torch.cat([t.reshape(-1) for p in eng.local_params() for t in p.values()]), ys)
        mesh.destroy()
    assert all(torch.equal(a.view(torch.int16), b.view(torch.int16)) for a, b in zip(out["rowmajor"][1], out["auto"][1]))
    assert torch.equal(out["rowmajor"][0].view(torch.int32), out["auto"][0].view(torch.int32))
    assert torch.isfinite(out["auto"][0]).all()
