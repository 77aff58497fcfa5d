"""TN GEMM ablation: MN-contiguous LDS-DMA loads vs transposed fragment reads (8192^3, bf16).

Historical (round 1, evidence for profiles/ablation_tn_r1_after.log): needs the ablation build of the GEMM
library at commit e72e569 (the ``ABL`` template parameter and ``dllm_gemm_ablation`` were removed from the
production library), loaded through ``DLLM_NATIVE_LIB=<path to that build>``."""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dllm  # noqa
import dllm._native as nat

n = 8192
A = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
B = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
C = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
L = nat.lib()
names = {0: "TN (mc loads, tr reads)", 3: "kc loads + tr reads", 12: "mc loads + kc reads", 15: "NT-like (kc/kc)",
         1: "A kc load only", 4: "A kc read only", 5: "A fully kc (=NN-like)", 10: "B fully kc"}
def run(abl):
    rc = L.dllm_gemm_ablation(abl, A.data_ptr(), B.data_ptr(), C.data_ptr(), n, torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc
res = {k: [] for k in names}
for _ in range(3):
    for k in names:
        run(k); torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            run(k)
        e.record(); torch.cuda.synchronize()
        res[k].append(s.elapsed_time(e) / 10)
for k, v in res.items():
    m = statistics.median(v)
    print(f"{names[k]:28s} {m:.3f} ms {2 * n**3 / m / 1e9:.0f} TF", flush=True)
