"""Per-launch durations of the kernels whose name contains a filter, from a rocprofv3 db.

usage: python tools/kern_durations.py DB FILTER [--skip N]
"""
import re
import sqlite3
import sys


def main():
    db, filt = sys.argv[1], sys.argv[2]
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    extra = [c for c in ("grid_x", "grid_y", "workgroup_x", "lds_size", "group_segment_size",
                         "grid_size_x", "grid_size_y", "workgroup_size_x") if c in cols]
    q = "select name, start, end" + "".join(", " + c for c in extra) + " from kernels order by start"
    for row in con.execute(q):
        n, s, e = row[:3]
        if filt in n:
            n = re.sub(r"\(anonymous namespace\)::", "", n)
            n = re.sub(r"\(.*", "", n)
            print(f"{(e - s) / 1e3:9.1f} us  " + " ".join(f"{c}={v}" for c, v in zip(extra, row[3:])) + f"  {n[:70]}")


if __name__ == "__main__":
    if len(sys.argv) < 3:
        print(__doc__)
        sys.exit(1)
    main()
