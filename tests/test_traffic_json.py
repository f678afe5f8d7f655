"""tools/traffic_json.py: per-launch traffic of the bench's roofline groups from PMC CSVs (CPU)."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _csv(d, counter, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for k, g, v in rows:
            w.writerow({"Kernel_Name": k, "Grid_Size": g, "Counter_Name": counter, "Counter_Value": v})


def test_groups_sum_and_average(tmp_path):
    vt, gm = "wino4_vt_kernel(Wino4Params)", "void conv_wino4_kernel<1>(Wino4Params)"
    # rocprofv3 spells the anonymous namespace out; the groups match without it
    zr0 = "void (anonymous namespace)::conv_wino5_kernel<0, 32, 2, 1>((anonymous namespace)::Wino5Params)"
    zr1 = "void conv_wino5_kernel<1, 32, 2, 1>(Wino5Params)"
    q0 = "void conv_wino5_kernel<0, 32, 1, 2>(Wino5Params)"
    ctx = "void conv_wino5_kernel<0, 32, 2, 0>(Wino5Params)"  # the context map: in no GRU group
    fetch = [(vt, 10, 100.0), (vt, 10, 300.0), (gm, 20, 1000.0), (gm, 20, 1000.0),
             (zr0, 5, 50.0), (zr1, 5, 70.0), (q0, 5, 40.0), (ctx, 5, 9999.0)]
    write = [(vt, 10, 400.0), (vt, 10, 400.0), (gm, 20, 30.0), (gm, 20, 50.0),
             (zr0, 5, 10.0), (zr1, 5, 10.0), (q0, 5, 20.0), (ctx, 5, 9999.0)]
    _csv(str(tmp_path / "f"), "FETCH_SIZE", fetch)
    _csv(str(tmp_path / "w"), "WRITE_SIZE", write)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic_json.py"),
                          str(tmp_path / "f"), str(tmp_path / "w"), "--batch", "16", "--size", "256"],
                         check=True, capture_output=True, text=True).stdout
    k = json.loads(out)["kernels"]
    # "sum" group: one logical launch = the transform launch + the GEMM launch
    assert k["conv_wino4"]["hbm_bytes_per_launch"] == int((2 * (200 + 1000) + (400 + 40)) * 1024)
    # averaged groups: FETCH doubled (gfx950 note), WRITE as is
    assert k["gru_zr"]["hbm_bytes_per_launch"] == int((2 * 60 + 10) * 1024)
    assert k["gru_q"]["hbm_bytes_per_launch"] == int((2 * 40 + 20) * 1024)
    assert k["conv_wino5_kernel_all"]["launches_fetch"] == 3
    assert "conv_wino_kernel<32,1>" not in k  # no such launches in the CSV
