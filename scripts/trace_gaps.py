"""Idle time of the GPU inside a rocprofv3 kernel trace (rocpd database, ``--kernel-trace -d DIR -o run``): over the
last ``--last_ms`` before the trace's last GEMM, the union of all kernels' busy intervals, the idle gaps between them (count and total
by size), and per kernel family the mean duration -- to tell a step that waits (gaps) from one whose kernels run
slower (interference), e.g. a method's normal steps against its collectives-elided steps (``bench.py
--elide_collectives``).

    python scripts/trace_gaps.py gpurun_out/prof/run_results.db [--last_ms 300]"""
import argparse
import collections
import sqlite3


def short(n: str, w: int = 64) -> str:
    return n.replace("void ", "").replace("dllm::", "")[:w]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last_ms", type=float, default=300.0)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute("select name, stream_id, start, end from kernels order by start").fetchall()
    rows = [r for r in rows if not short(r[0]).startswith("stamp_kernel")]
    t_end = max(r[3] for r in rows if "gemm" in r[0])   # the last GEMM: ignore teardown / readout kernels
    cut = t_end - a.last_ms * 1e6
    rows = [r for r in rows if r[2] >= cut and r[3] <= t_end]
    busy, last, gaps = 0, rows[0][2], []
    for _, _, s, e in rows:
        if s > last:
            gaps.append(s - last)
        s = max(s, last)
        if e > s:
            busy += e - s
            last = e
    span = last - rows[0][2]
    print(f"window {span / 1e6:.2f} ms, kernels {len(rows)}, busy {busy / 1e6:.2f} ms ({100 * busy / span:.2f} %), "
          f"idle {(span - busy) / 1e6:.3f} ms in {len(gaps)} gaps")
    for lo, hi in ((0, 5e3), (5e3, 20e3), (20e3, 100e3), (100e3, 1e12)):
        g = [x for x in gaps if lo <= x < hi]
        print(f"  gaps {lo / 1e3:>5.0f}-{hi / 1e3 if hi < 1e12 else float('inf'):>5.0f} us: {len(g):5d}  total "
              f"{sum(g) / 1e6:.3f} ms")
    fam = collections.defaultdict(list)
    per_stream = collections.defaultdict(float)
    for n, st, s, e in rows:
        fam[short(n)].append(e - s)
        per_stream[st] += e - s
    print(f"{'n':>5s} {'mean_us':>9s} {'total_ms':>9s}  kernel")
    for n, v in sorted(fam.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):5d} {sum(v) / len(v) / 1e3:9.1f} {sum(v) / 1e6:9.2f}  {n}")
    print("kernel ms per stream:", {k: round(v / 1e6, 2) for k, v in sorted(per_stream.items())})


if __name__ == "__main__":
    main()
