"""Which hardware queue / stream each kernel family ran on, from a rocprofv3 rocpd database (``--kernel-trace -d DIR
-o run``): the evidence for the compute-queue reservation (utils/streams.py) -- compute-stream GEMMs and the side /
collective streams' kernels must not share a queue id.

    python scripts/queue_ids.py gpurun_out/prof/run_results.db [--skip_probe]"""
import argparse
import collections
import sqlite3


def short(n: str, w: int = 70) -> str:
    return n.replace("void ", "").replace("dllm::", "")[:w]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute("select name, queue_id, stream_id, duration from kernels").fetchall()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for name, q, s, dur in rows:
        if short(name).startswith("stamp_kernel"):
            continue   # the reservation's own probe kernels
        k = (q, s, short(name))
        agg[k][0] += 1
        agg[k][1] += dur / 1e3
    print(f"{'hw-queue':>8s} {'stream':>6s} {'n':>5s} {'mean_us':>9s}  kernel")
    for (q, s, n), (c, us) in sorted(agg.items(), key=lambda kv: (kv[0][0], kv[0][1], -kv[1][1])):
        print(f"{q:>8} {s:>6} {c:>5d} {us / c:>9.1f}  {n}")
    byq = collections.defaultdict(set)
    for (q, s, n) in agg:
        byq[q].add(s)
    print("\nstreams per hardware queue:", {q: sorted(v) for q, v in sorted(byq.items())})


if __name__ == "__main__":
    main()
