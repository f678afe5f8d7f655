"""The bench's headline roofline recomputed from a committed rocprofv3 kernel-trace summary.

usage: python tools/trace_roofline.py profiles/r05/prof_p_stats_c1.txt --batch 16 --size 256
       python tools/trace_roofline.py profiles/r05/prof_p_stats_c4.txt --batch 32 --size 512

The headline kernel is conv_wino5_kernel over the SepConvGRU's four launches of an iteration
(bench.py): z|r (EPI 1: both stages) and q (EPI 2: both stages).  achieved = Σ executed FLOPs of
one z|r and one q launch ÷ Σ their mean durations, each mean taken over the 1×5 and 5×1
launches from the trace's per-kernel averages (stats_file.py format: calls, total ms, avg µs,
pct, kernel).  Executed FLOPs as bench.py / ConvRunner.mfma_flops: 8 transform points per
4-pixel tile, K = h (or r·h) 128 + motion 128, N = 256 (z|r) or 128 (q), channels padded to 32.
"""
import argparse
import re

PEAK_TFLOPS = 157.3  # MI355X fp32 MFMA (MI355X_MICROARCH.md), as bench.py


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    a = ap.parse_args()
    m_px = a.batch * (a.size // 8) ** 2
    durs = {1: [], 2: []}
    for line in open(a.stats):
        m = re.match(r"\s*(\d+)\s+([\d.]+)\s+([\d.]+)\s+[\d.]+\s+.*conv_wino5_kernel<(\d), (\d+), (\d), (\d)>", line)
        if m and int(m.group(7)) in durs:
            durs[int(m.group(7))].append(float(m.group(3)))
    if not durs[1] or not durs[2]:
        raise SystemExit("no GRU z|r / q launches in " + a.stats)
    zr_us, q_us = sum(durs[1]) / len(durs[1]), sum(durs[2]) / len(durs[2])
    k = 128 + 128
    fl_zr = 2.0 * 8 * (m_px / 4) * k * 256
    fl_q = 2.0 * 8 * (m_px / 4) * k * 128
    ach = (fl_zr + fl_q) / ((zr_us + q_us) * 1e-6) / 1e12
    print(f"z|r {zr_us:.2f} us, q {q_us:.2f} us (trace means over both stages) -> "
          f"{ach:.2f} TFLOP/s executed = {ach / PEAK_TFLOPS:.4f} of {PEAK_TFLOPS} TFLOP/s")


if __name__ == "__main__":
    main()
