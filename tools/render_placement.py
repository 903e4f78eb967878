"""Where the overlapped render's kernels run inside the bench frame, from a
rocprofv3 kernel trace of bench.py (GPU diagnostic): for the last two whole
frames, each render kernel's start and end relative to the frame start (the
k_postprocess before it), beside the re-binning launches (k_finish_bins:
the graph segment boundaries) and whether a simulator kernel ran at the
same time.

    python3 tools/render_placement.py run_kernel_trace.csv
"""
import csv
import sys

SIM = ("k_fused", "k_grid_f", "k_finish_bins", "k_bin", "k_permute")


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    posts = [a for a, b, n in ks if "k_postprocess" in n]
    t0, t1, t2 = posts[-3], posts[-2], posts[-1]
    short = lambda n: n.split("(")[0].replace("gsmpm::", "").replace("void ", "")[:22]
    for f0, f1 in ((t0, t1), (t1, t2)):
        win = [(a, b, n) for a, b, n in ks if a >= f0 and a < f1]
        sims = [(a, b) for a, b, n in win if any(s in n for s in SIM)]
        bins = [round((a - f0) / 1e3, 1) for a, b, n in win if "k_finish_bins" in n]
        print(f"frame {(f1 - f0) / 1e3:.1f} us; re-binnings at {bins} us")
        for a, b, n in win:
            if "gsmpm::" not in n or any(s in n for s in SIM) or "k_postprocess" in n or "k_world" in n:
                continue
            beside = sum(1 for c, d in sims if c < b and d > a)
            print(f"  {short(n):22s} {(a - f0) / 1e3:8.1f} -> {(b - f0) / 1e3:8.1f} us  beside {beside} sim kernels")


if __name__ == "__main__":
    main(sys.argv[1])
