"""Per-kernel summary of a rocprofv3 kernel trace (run_kernel_trace.csv):
launches, mean, median, and the mean without each kernel's first launch
(the code-object load / first graph replay) -- the figure bench.py's
packet-stamped average is compared with.  Kernels are grouped by the name
up to its template arguments' closing '>' (k_fused<0, 7> etc.).

    python3 tools/trace_summary.py run_kernel_trace.csv
"""
import csv
import statistics
import sys


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("gsmpm::", "")


def main(path):
    rows = list(csv.DictReader(open(path)))
    if not rows:
        print("empty trace")
        return
    kn = next(k for k in rows[0] if "Kernel_Name" in k)
    t0 = next(k for k in rows[0] if "Start_Timestamp" in k)
    t1 = next(k for k in rows[0] if "End_Timestamp" in k)
    by = {}
    for r in rows:
        by.setdefault(short(r[kn]), []).append((int(r[t0]), int(r[t1]) - int(r[t0])))
    tot = sum(d for v in by.values() for _, d in v)
    print(f"{'kernel':40s} {'calls':>6s} {'mean_us':>9s} {'median_us':>9s} {'mean_wo_first':>13s} {'share':>6s}")
    for k, v in sorted(by.items(), key=lambda kv: -sum(d for _, d in kv[1])):
        v.sort()
        ds = [d / 1e3 for _, d in v]
        rest = ds[1:] or ds
        s = sum(ds) * 1e3
        print(f"{k[:40]:40s} {len(ds):6d} {statistics.mean(ds):9.2f} {statistics.median(ds):9.2f} "
              f"{statistics.mean(rest):13.2f} {s / tot:6.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
