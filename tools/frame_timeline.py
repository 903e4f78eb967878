"""Where a bench frame's time goes, from a rocprofv3 kernel trace of bench.py
(tools/gpu_r04n.sh): for the timed frames, the simulator's kernels (k_fused,
k_grid_f, binning) with and without a render kernel running beside them.

    python3 tools/frame_timeline.py run_kernel_trace.csv
"""
import csv
import sys

SIM = ("k_fused", "k_grid_f", "k_finish_bins", "k_bin", "k_permute")
POST = ("k_postprocess", "k_world_out")


def kind(name):
    if any(s in name for s in SIM):
        return "sim"
    if any(s in name for s in POST):
        return "post"
    if "gsmpm::" in name:
        return "render"
    return "other"


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # the last 6 postprocess launches delimit the last frames
    posts = [a for a, b, n in ks if "k_postprocess" in n]
    if len(posts) < 4:
        print("too few frames in the trace")
        return
    t0, t1 = posts[-4], posts[-1]  # three whole frames
    win = [(a, b, n, kind(n)) for a, b, n in ks if a >= t0 and b <= t1]
    rend = [(a, b) for a, b, n, k in win if k == "render"]
    tot = {"sim": 0, "post": 0, "render": 0, "other": 0}
    for a, b, n, k in win:
        tot[k] += b - a
    # sim kernels overlapped by a render kernel: their durations
    ov, alone = [], []
    for a, b, n, k in win:
        if k != "sim" or "k_fused<0, 3>" not in n:
            continue
        hit = any(c < b and d > a for c, d in rend)
        (ov if hit else alone).append(b - a)
    span = (t1 - t0) / 3
    print(f"frame {span / 1e3:.1f} us (3 frames); kernel time per frame: sim {tot['sim'] / 3e3:.1f} us, "
          f"post {tot['post'] / 3e3:.1f}, render {tot['render'] / 3e3:.1f}")
    if ov and alone:
        print(f"k_fused<0,3>: {len(alone)} launches alone, mean {sum(alone) / len(alone) / 1e3:.2f} us; "
              f"{len(ov)} beside a render kernel, mean {sum(ov) / len(ov) / 1e3:.2f} us")
        # per render kernel: the k_fused / k_grid_f launches it overlapped and their extra time
        base = {"k_fused<0, 3>": sum(alone) / len(alone)}
        g_alone = [b - a for a, b, n, k in win if "k_grid_f" in n and not any(c < b and d > a for c, d in rend)]
        if g_alone:
            base["k_grid_f"] = sum(g_alone) / len(g_alone)
        short = lambda n: n.split("(")[0].replace("gsmpm::", "").replace("void ", "")
        per = {}
        for c, d, rn, rk in win:
            if rk != "render":
                continue
            e = per.setdefault(short(rn), {"launches": 0, "us": 0.0, "sim_overlapped": 0, "sim_extra_us": 0.0})
            e["launches"] += 1
            e["us"] += (d - c) / 1e3
            for a, b, n, k in win:
                sn = next((x for x in base if x in n), None)
                if sn and c < b and d > a:
                    e["sim_overlapped"] += 1
                    e["sim_extra_us"] += (b - a - base[sn]) / 1e3
        print("per render kernel, 3 frames: launches, own time, sim launches beside it, their extra time "
              "over the alone mean (a sim launch beside two render kernels counts for both)")
        for nm, e in sorted(per.items(), key=lambda kv: -kv[1]["sim_extra_us"]):
            print(f"  {nm:<22} {e['launches']:3d}  {e['us']:8.1f} us  {e['sim_overlapped']:4d}  {e['sim_extra_us']:8.1f} us")
    # idle: gaps in the union of all kernel intervals
    busy, cur_a, cur_b = 0, None, None
    for a, b, n, k in win:
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                busy += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        busy += cur_b - cur_a
    print(f"GPU busy (any kernel) {busy / 3e3:.1f} us per frame, idle {(t1 - t0 - busy) / 3e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
