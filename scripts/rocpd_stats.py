"""Summarise a rocprofv3 rocpd database (``-d DIR -o run`` -> ``DIR/run_results.db``): per-kernel totals, plus
a steady-state timeline of the last step(s).

    python scripts/rocpd_stats.py gpurun_out/prof/run_results.db [--last_ms 30.6] [--timeline N]

``--last_ms``: also print every dispatch of the final window of that length (one step), with gaps."""
import argparse
import collections
import sqlite3


def short(n: str, w: int = 88) -> str:
    n = n.replace("void ", "").replace("dllm::", "")
    return n[:w]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last_ms", type=float, default=0.0)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--overlap", default="",
                    help="comma substrings of communication kernels (e.g. 'copyBuffer,nccl'): over the whole trace after the "
                         "first --skip_ms, report the union of their intervals and the part under GEMM kernels "
                         "('gemm_'), i.e. the trace's own overlap_frac to compare with the comm observer")
    ap.add_argument("--skip_ms", type=float, default=0.0)
    ap.add_argument("--from_marker", type=int, default=0,
                    help="--overlap window starts at the K-th last step start (--step_marker, draws 2 per step): "
                         "the window a CommObserver over the last K steps of the same process saw")
    ap.add_argument("--step_marker", default="",
                    help="substring of the kernel that starts a step (e.g. 'rng_normal_kernel<unsigned short>'): "
                         "print the timeline of the second-to-last complete step instead of --last_ms")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
    agg = collections.defaultdict(lambda: [0, 0])
    for n, s, e, *_ in rows:
        agg[n][0] += 1
        agg[n][1] += e - s
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':88s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'%':>6s}")
    for n, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{short(n):88s} {k:6d} {t / k / 1e3:9.1f} {t / 1e6:9.2f} {100 * t / tot:6.2f}")
    print(f"total kernel time {tot / 1e6:.2f} ms over {len(rows)} dispatches")
    if a.overlap and rows:
        keys = a.overlap.split(",")
        t_lo = rows[0][1] + a.skip_ms * 1e6
        if a.last_ms > 0:  # steady state: the final window only
            t_lo = max(t_lo, max(r[2] for r in rows) - a.last_ms * 1e6)
        if a.from_marker and a.step_marker:
            starts = [r[1] for r in rows if a.step_marker in r[0]][::2]
            t_lo = max(t_lo, starts[-a.from_marker])

        def union(iv):
            out = []
            for s_, e_ in sorted(iv):
                if out and s_ <= out[-1][1]:
                    out[-1][1] = max(out[-1][1], e_)
                else:
                    out.append([s_, e_])
            return out

        comm = union([(s_, e_) for n, s_, e_, *_ in rows if s_ >= t_lo and any(k in n for k in keys)])
        gem = union([(s_, e_) for n, s_, e_, *_ in rows if s_ >= t_lo and "gemm_" in n])
        hid, i, j = 0, 0, 0
        while i < len(comm) and j < len(gem):
            lo, hi = max(comm[i][0], gem[j][0]), min(comm[i][1], gem[j][1])
            hid += max(0, hi - lo)
            if comm[i][1] < gem[j][1]:
                i += 1
            else:
                j += 1
        un = sum(e_ - s_ for s_, e_ in comm)
        print(f"\ncomm kernels {keys}: union {un / 1e6:.3f} ms, under GEMMs {hid / 1e6:.3f} ms, "
              f"overlap_frac {hid / un if un else float('nan'):.3f}")
    if a.step_marker and rows:
        # step period over the trace's last steps: start-to-start, and the idle time before each step's first kernel
        # (nothing of the previous step still running: a host that cannot keep the queue fed)
        st = [i for i, r in enumerate(rows) if a.step_marker in r[0]][::2]
        per, idle = [], []
        for i0, i1 in list(zip(st[:-1], st[1:]))[-40:]:
            per.append(rows[i1][1] - rows[i0][1])
            idle.append(max(0, rows[i1][1] - max(r[2] for r in rows[i0:i1])))
        if per:
            per.sort()
            idle.sort()
            print(f"\nsteps {len(per)}: period median {per[len(per) // 2] / 1e3:.1f} us (min {per[0] / 1e3:.1f}, max "
                  f"{per[-1] / 1e3:.1f}); idle before the step median {idle[len(idle) // 2] / 1e3:.1f} us")
    win = []
    if a.step_marker and rows:
        starts = [i for i, r in enumerate(rows) if a.step_marker in r[0]]
        # the marker may occur several times per step (x and dy draws): steps start at every other one
        if len(starts) >= 6:
            i0, i1 = starts[-6], starts[-4]
            win = rows[i0:i1]
    elif a.last_ms > 0 and rows:
        t1 = max(r[2] for r in rows)
        cut = t1 - a.last_ms * 1e6
        win = [r for r in rows if r[1] >= cut]
    if win:
        busy, last = 0, 0
        print(f"\nwindow: {len(win)} dispatches")
        for n, s, e, gx, wx in win:
            gap = (s - last) / 1e3 if last else 0.0
            print(f"  +{(s - win[0][1]) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap:7.1f}  grid {gx // max(wx, 1):6d}  {short(n, 70)}")
            busy += max(0, e - max(s, last))
            last = max(last, e)
        span = win[-1][2] - win[0][1]
        print(f"window span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f}%)")


if __name__ == "__main__":
    main()
