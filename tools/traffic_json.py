"""Per-launch HBM-side traffic of the bench's roofline kernel from two rocprofv3 PMC passes.

usage: python tools/traffic_json.py FETCH_DIR WRITE_DIR SUBSTRING [SUBSTRING ...] > profiles/traffic_gru_zr.json

Kernels whose name contains any SUBSTRING (e.g. the 1×5 and 5×1 z|r launches) are averaged.
FETCH_SIZE is doubled per MI355X_MICROARCH.md's gfx950 note (16-B-per-lane reads are tallied at
64 B per 128-B request); WRITE_SIZE is taken as is; both are KiB, memory side of L2.
"""
import collections
import csv
import glob
import json
import sys


def per_kernel(d, counter):
    path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    fdir, wdir, subs = sys.argv[1], sys.argv[2], sys.argv[3:]
    fetch, write = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    pick = lambda d: {k: v for k, v in d.items() if any(s in k for s in subs)}  # noqa: E731
    f, w = pick(fetch), pick(write)
    fk = {k[:70]: sum(v) / len(v) for k, v in f.items()}
    wk = {k[:70]: sum(v) / len(v) for k, v in w.items()}
    favg = sum(sum(v) for v in f.values()) / sum(len(v) for v in f.values())
    wavg = sum(sum(v) for v in w.values()) / sum(len(v) for v in w.values())
    m = 16 * 32 * 32
    alg = 4 * m * (256 + 256 + 128 + 256) + 4 * 256 * 256 * 5  # in h|motion, bias map, h, z|rh out, W
    print(json.dumps({
        "kernel": " + ".join(subs) + " (launches averaged)", "batch": 16, "size": 256,
        "hbm_bytes_per_launch": int((2 * favg + wavg) * 1024),
        "fetch_size_kb_raw": fk, "write_size_kb": wk,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py "
                  "--steps 2 --warmup 1 (decoder only); FETCH_SIZE doubled per the gfx950 note; "
                  "WRITE_SIZE as is; memory-side (L2->fabric) bytes, Infinity-Cache hits included",
        "algorithmic_bytes_per_launch": alg}, indent=1))


if __name__ == "__main__":
    main()
