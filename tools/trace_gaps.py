"""Kernel-trace timeline of the substep kernels (rocprofv3 --kernel-trace CSV):
per-kernel duration and the idle gap before each launch, over the longest
run of back-to-back substep kernels (one graph replay).  Usage:
    python tools/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv"""
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.split("(")[0].replace("void ", "").replace("gsmpm::", "")[:28]
sub = [r for r in rows if any(k in r["Kernel_Name"] for k in ("k_fused", "k_grid", "k_p2g", "k_g2p", "k_finish_bins",
                                                                "k_scan", "k_scatter"))]
dur, gap = defaultdict(list), defaultdict(list)
for a, b in zip(sub, sub[1:]):
    g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    if g < 50:  # inside one graph replay
        gap[short(b["Kernel_Name"])].append(g)
for r in sub:
    dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
med = lambda v: sorted(v)[len(v) // 2]
print(f"{'kernel':30s} {'n':>6s} {'dur med us':>10s} {'dur mean':>9s} {'gap-before med':>14s} {'gap mean':>9s}")
for k in dur:
    print(f"{k:30s} {len(dur[k]):6d} {med(dur[k]):10.2f} {sum(dur[k])/len(dur[k]):9.2f} "
          f"{med(gap[k]) if gap[k] else float('nan'):14.2f} {sum(gap[k])/max(1,len(gap[k])):9.2f}")

# frame spans: consecutive kernels (any) separated by < 20 us idle form one burst
bursts, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 20000:
        bursts.append(cur)
        cur = []
    cur.append(b)
bursts.append(cur)
print("\nbursts (>= 50 kernels): span us, busy us, kernels; idle before next")
for i, bu in enumerate(bursts):
    if len(bu) < 50:
        continue
    span = (int(bu[-1]["End_Timestamp"]) - int(bu[0]["Start_Timestamp"])) / 1e3
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in bu) / 1e3
    nxt = (int(bursts[i + 1][0]["Start_Timestamp"]) - int(bu[-1]["End_Timestamp"])) / 1e3 if i + 1 < len(bursts) else 0
    print(f"  {span:9.1f} {busy:9.1f} {len(bu):5d}   idle after {nxt:9.1f}")
# the non-substep kernels of the last burst
last = [b for b in bursts if len(b) >= 50][-1]
other = defaultdict(float)
for r in last:
    k = short(r["Kernel_Name"])
    if not any(s in k for s in ("k_fused", "k_grid", "k_finish")):
        other[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("  other kernels in the last burst (us):", {k: round(v, 1) for k, v in other.items()})
