"""Per-launch memory-side traffic of the bench's roofline kernels from two rocprofv3 PMC passes.

usage: python tools/traffic_json.py FETCH_DIR WRITE_DIR --batch B --size S [--iters I]
           > profiles/traffic_<tag>.json

For every kernel group below (kernel-name substrings), the counters of its launches are averaged:
FETCH_SIZE is doubled per MI355X_MICROARCH.md's gfx950 note (16-B-per-lane reads are tallied at
64 B per 128-B request); WRITE_SIZE is taken as is; both are KiB on the memory side of L2
(Infinity-Cache hits included).  Each group also carries its ALGORITHMIC bytes per launch
(compulsory reads + writes) and the ratio counter / algorithmic — well above 1
means re-reads.
"""
import argparse
import collections
import csv
import glob
import json
import re


def groups(B, S):
    h = w = S // 8
    M = B * h * w
    P = h * w
    f = 4
    heads = f * (M * 128 + M * 512 + 512 * 128 * 9)            # XHead hidden convs 128→512
    corr1 = f * (M * 256 + M * 192 + 192 * 256 * 9)            # corr_net.1 256→192
    # SepConvGRU, context hoisted (K = h or r·h 128 + motion 128): z|r reads h|motion and its
    # bias-map slice (256 ch), writes z and r·h; q reads r·h|motion, its bias-map slice (128),
    # z and h, writes h; weights 5 taps each
    zr = f * M * (256 + 256 + 256) + f * 256 * 256 * 5
    q = f * M * (256 + 128 + 128 + 128 + 128) + f * 128 * 256 * 5
    lookup = B * (4 * P * sum(min(100, P // 4 ** l) for l in range(4)) + 4 * P * 324)
    pose_step = B * 36 * S * S
    lookup_conv = B * (4 * P * sum(min(100, P // 4 ** l) for l in range(4)) + 4 * P * 256) + 4 * 328 * 256
    # the critical-path ↓8 launch (parts = 2): the pose flow at the 4 bilinear source pixels of
    # every feature pixel (4 × 16-B points) + the next iteration's ↓8 flow (F2 and HX, 2 × 8 B)
    pose_step_crit = M * (4 * 16 + 16)

    def conv(cin, cout, taps=9):
        return f * (M * cin + M * cout + cout * cin * taps)
    small = [conv(256, 126), conv(128, 64), conv(128, 64), conv(64, 32)]  # the <32,1> launches
    return {
        "conv_wino5_kernel_all": ([", 1>(Wino5Params", ", 2>(Wino5Params"], (zr + q) / 2,
                                  "F(4,5) Winograd, every SepConvGRU launch of an iteration (z|r "
                                  "and q of both stages, launches averaged)"),
        # template <DIR, W, NBW, EPI>: EPI 1 = GRU_ZR, 2 = GRU_Q (0: the per-forward context map)
        "gru_zr": ([", 1>(Wino5Params"], zr,
                   "SepConvGRU z|r 1×5 + 5×1 (context hoisted)"),
        "gru_q": ([", 2>(Wino5Params"], q,
                  "SepConvGRU q 1×5 + 5×1 (context hoisted)"),
        "conv_wino4": (["wino4_vt_kernel", "conv_wino4_kernel<"], (heads + corr1) / 2,
                       "F(4×4,3×3) Winograd: XHead hidden 128→512 + corr_net.1 256→192; one launch "
                       "= the transform launch + the point-GEMM launch (their averages summed; "
                       "the transformed input V round-trips through memory between them)", "sum"),
        "conv_wino_kernel<32,1>": (["conv_wino_kernel<32, 1>"], sum(small) / 4,
                                   "F(2x2,3x3) Winograd <32,1>: out_net 256→126, flow_net.1 / "
                                   "delta_flow_encoder.1 128→64, mask_encoder.1 64→32"),
        "conv_wino_kernel<64,*>": (["conv_wino_kernel<64, 2>", "conv_wino_kernel<64, 1>"], sum(small) / 4,
                                   "F(2x2,3x3) Winograd at 64-wide maps (configs[4]): out_net 256→126, "
                                   "flow_net.1 / delta_flow_encoder.1 128→64 <64,2>, mask_encoder.1 "
                                   "64→32 <64,1> (launches averaged)"),
        "conv_wino_kernel": (["conv_wino_kernel<32, 2>", "conv_wino_kernel<32, 3>"], (heads + corr1) / 2,
                             "F(2x2,3x3) Winograd <32,2> / <32,3> (only with SCFLOW_CONV_WINO4=0): "
                             "XHead hidden 128→512 + corr_net.1 256→192 (launches averaged)"),
        "corr_lookup": (["corr_lookup_lds_kernel"], lookup, "pyramid lookup r=4, 4 levels"),
        "corr_lookup_conv": (["corr_lookup_conv1x1_kernel"], lookup_conv, "pyramid lookup fused "
                             "into corr_net.0: window reads + 256-channel output + weights"),
        "pose_step": (["pose_step_kernel"], pose_step, "pose update + pose flow + ×8 flow/mask "
                      "(every launch kind averaged: use the two entries below)"),
        "pose_step_fullres": (["pose_step_kernel"], pose_step, "pose_step_kernel, its deferred "
                              "full-resolution launch only (7 per forward): pose flow + ×8 "
                              "flow/mask, 36 B per full-resolution pixel", "wide"),
        "pose_step_crit": (["pose_step_kernel"], pose_step_crit, "pose_step_kernel, its critical-"
                           "path ↓8 launch only (the smallest grid): pose update + the next "
                           "iteration's ↓8 flow, 80 B per feature pixel", "min"),
    }


def per_kernel(d, counter):
    """{kernel name: [(grid size, counter value) per launch]}"""
    path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
            vals[name].append((int(r.get("Grid_Size") or 0), float(r["Counter_Value"])))
    return vals


def select(vals, subs, which):
    """Counter values of the launches of kernels matching ``subs``; ``which`` keeps one launch
    kind: "min" the launches with the smallest grid, "wide" those with the most frequent grid size
    above the smallest (the pose step: 7 deferred full-resolution launches per forward at B × 64
    workgroups vs the last iteration's single combined launch, whose grid is larger still)."""
    got = [gv for k, vs in vals.items() if any(s in k for s in subs) for gv in vs]
    if which and got:
        lo = min(g for g, _ in got)
        if which == "min":
            pick = lo
        else:
            above = collections.Counter(g for g, _ in got if g > lo)
            pick = above.most_common(1)[0][0] if above else lo
        got = [gv for gv in got if gv[0] == pick]
    return [v for _, v in got]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--iters", type=int, default=8)
    a = ap.parse_args()
    fetch, write = per_kernel(a.fetch_dir, "FETCH_SIZE"), per_kernel(a.write_dir, "WRITE_SIZE")
    out = {"batch": a.batch, "size": a.size, "iters": a.iters,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     "bench.py (decoder leg only); FETCH_SIZE doubled per the gfx950 note; "
                     "WRITE_SIZE as is; memory-side (L2->fabric) bytes, Infinity-Cache hits included",
           "kernels": {}}
    for name, (subs, alg, what, *which) in groups(a.batch, a.size).items():
        mode = which[0] if which else None
        if mode == "sum":  # one logical launch = one launch of each kernel in ``subs``
            fs = [select(fetch, [s], None) for s in subs]
            ws = [select(write, [s], None) for s in subs]
            if not all(fs) or not all(ws):
                continue
            f = [sum(sum(v) / len(v) for v in fs)]
            w = [sum(sum(v) / len(v) for v in ws)]
        else:
            f = select(fetch, subs, mode)
            w = select(write, subs, mode)
        if not f or not w:
            continue
        hbm = (2 * sum(f) / len(f) + sum(w) / len(w)) * 1024
        out["kernels"][name] = {
            "what": what, "match": subs, "launches_fetch": len(f), "launches_write": len(w),
            "hbm_bytes_per_launch": int(hbm),
            "fetch_kb_raw_avg": round(sum(f) / len(f), 1), "write_kb_avg": round(sum(w) / len(w), 1),
            "algorithmic_bytes_per_launch": int(alg), "ratio_to_algorithmic": round(hbm / alg, 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
