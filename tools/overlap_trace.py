"""Overlap of the slab window exchange with the interior grid pass, from one
rank's rocprofv3 kernel trace (tools/gpu_r04f.sh runs a 2-rank RCCL slab bench,
every rank under its own rocprofv3 --kernel-trace).

Per substep a slab rank launches k_fused, k_grid_f over the window tiles
(pass 1), then -- inside the captured graph, on a forked branch -- k_grid_f
over the interior tiles (pass 2) while the RCCL group (ncclDevKernel_*)
swaps the window partials, then k_win_update.  This reads the trace's
begin/end stamps and reports how much of each exchange kernel's interval the
interior pass covers.

    python3 tools/overlap_trace.py path/to/run_kernel_trace.csv
"""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    grid = [(a, b) for a, b, n in ks if "k_grid_f" in n]
    nccl = [(a, b) for a, b, n in ks if "nccl" in n.lower()]
    fused = [a for a, b, n in ks if "k_fused" in n]
    # the interior pass: the second k_grid_f after each k_fused
    interior = []
    fi = 0
    seen = 0
    for a, b in grid:
        while fi < len(fused) and fused[fi] < a:
            fi += 1
            seen = 0
        seen += 1
        if seen == 2:
            interior.append((a, b))
    tot = cov = 0
    concurrent = 0
    for a, b in nccl:
        tot += b - a
        o = 0
        for c, d in interior:
            if d <= a:
                continue
            if c >= b:
                break
            o += min(b, d) - max(a, c)
        cov += o
        concurrent += 1 if o > 0 else 0
    print(f"kernels {len(ks)}, k_grid_f {len(grid)} (interior {len(interior)}), exchange kernels {len(nccl)}")
    if nccl:
        print(f"exchange kernels overlapping an interior pass: {concurrent} of {len(nccl)}; "
              f"exchange time {tot / 1e3:.1f} us, of it under an interior pass {cov / 1e3:.1f} us "
              f"({100.0 * cov / max(tot, 1):.1f} %)")
    if interior:
        it = sum(b - a for a, b in interior)
        under = 0
        for c, d in interior:
            for a, b in nccl:
                if b <= c:
                    continue
                if a >= d:
                    break
                under += min(b, d) - max(a, c)
        print(f"interior pass time {it / 1e3:.1f} us total, {it / len(interior) / 1e3:.2f} us each; "
              f"under an exchange kernel {under / 1e3:.1f} us ({100.0 * under / max(it, 1):.1f} %)")
    # the window pass (first k_grid_f after each k_fused) to the next exchange kernel's start
    gaps = []
    fi = seen = 0
    for a, b in grid:
        while fi < len(fused) and fused[fi] < a:
            fi += 1
            seen = 0
        seen += 1
        if seen == 1:
            nxt = next((x for x, _ in nccl if x >= a), None)
            if nxt is not None and nxt - b < 5e5:
                gaps.append(nxt - b)
    if gaps:
        gaps.sort()
        print(f"window pass end -> exchange kernel start: median {gaps[len(gaps) // 2] / 1e3:.2f} us over {len(gaps)}")
    # off the critical path: interior-pass time inside [its window pass's end, the next exchange kernel's end]
    # (the exchange -- RCCL's launch and its kernel -- follows the window pass; k_win_update waits for both)
    hid = tot_i = 0
    wins = []
    fi = seen = 0
    for a, b in grid:
        while fi < len(fused) and fused[fi] < a:
            fi += 1
            seen = 0
        seen += 1
        if seen == 1:
            wins.append(b)
    for c, d in interior:
        w_end = max((x for x in wins if x <= c), default=None)
        x_end = next((e for x, e in nccl if x >= (w_end if w_end is not None else c)), None)
        tot_i += d - c
        if w_end is not None and x_end is not None:
            hid += max(0, min(d, x_end) - max(c, w_end))
    if tot_i:
        print(f"interior pass time between its window pass's end and the exchange kernel's end: "
              f"{100.0 * hid / tot_i:.1f} % (off the critical path)")


if __name__ == "__main__":
    main(sys.argv[1])
