"""Summarise a rocprofv3 kernel_stats.csv / kernel_trace.csv pair (per-kernel totals and busy fraction)."""
import csv, sys, collections

def short(n):
    n = n.replace("void ", "").replace("dllm::", "")
    return n[:90]

d = sys.argv[1]
rows = list(csv.DictReader(open(f"{d}/k_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'kernel':90s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'%':>6s}")
for r in rows[:25]:
    print(f"{short(r['Name']):90s} {r['Calls']:>6s} {float(r['AverageNs'])/1e3:9.1f} "
          f"{float(r['TotalDurationNs'])/1e6:9.2f} {float(r['Percentage']):6.2f}")
tr = list(csv.DictReader(open(f"{d}/k_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
if len(sys.argv) > 2:  # window: last fraction of the trace
    frac = float(sys.argv[2])
    t0 = int(tr[0]["Start_Timestamp"]); t1 = max(int(r["End_Timestamp"]) for r in tr)
    cut = t1 - frac * (t1 - t0)
    tr = [r for r in tr if int(r["Start_Timestamp"]) >= cut]
busy = 0; last = 0
for r in tr:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    s = max(s, last)
    if e > s: busy += e - s; last = max(last, e)
span = int(tr[-1]["End_Timestamp"]) - int(tr[0]["Start_Timestamp"])
print(f"window span {span/1e6:.2f} ms, busy {busy/1e6:.2f} ms ({100*busy/span:.1f}%), kernels {len(tr)}")
