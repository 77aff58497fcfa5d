"""Device mock-data RNG throughput (Philox4x32-10 + Box-Muller) on the flagship batch shape [8192, 4096]."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dllm  # noqa
from dllm.ops.elementwise import rng_normal_

for dt in (torch.bfloat16, torch.float32):
    t = torch.empty(8192, 4096, dtype=dt, device="cuda")
    for _ in range(3):
        rng_normal_(t, seed=1)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(50):
        rng_normal_(t, seed=i)
    e.record(); torch.cuda.synchronize()
    us = s.elapsed_time(e) / 50 * 1e3
    print(f"rng {dt}: {us:.1f} us per [8192, 4096] ({t.numel() * t.element_size() / us / 1e6:.2f} TB/s)", flush=True)
