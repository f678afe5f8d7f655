"""Per-iteration kernel timeline from a rocprofv3 kernel-trace db (both streams).

usage: python tools/timeline.py DB [--iteration I] [--marker NAME]
Finds SCFlowDecoder iterations by a marker kernel that starts every iteration once (default the
pyramid lookup) and prints, for one iteration (marker I to marker I+1), every kernel: start
offset, duration, stream, gap to the previous kernel on any stream; then the iteration's wall
time, busy time (union of kernel intervals) and idle gaps.
"""
import argparse
import re
import sqlite3


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*", "", n)
    return n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--iteration", type=int, default=20, help="global index of the iteration")
    ap.add_argument("--marker", default="corr_lookup", help="kernel-name substring starting an iteration")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = list(con.execute("select name, start, end, stream_id, queue_id from kernels order by start"))
    starts = [i for i, r in enumerate(rows) if a.marker in r[0]]
    it = a.iteration
    lo, hi = starts[it], starts[it + 1]
    seg = rows[lo:hi]
    t0 = seg[0][1]
    busy_end = t0
    busy = 0
    idle = []
    for name, s, e, st, q in seg:
        gap = s - busy_end
        if gap > 0:
            idle.append(gap)
        print(f"{(s - t0) / 1e3:8.2f} us  dur {(e - s) / 1e3:7.2f}  q{q}  gap {max(gap, 0) / 1e3:6.2f}  {short(name)}")
        if e > busy_end:
            busy += e - max(s, busy_end)
            busy_end = e
    wall = seg[-1][2] - t0
    print(f"iteration wall {wall / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {sum(idle) / 1e3:.1f} us "
          f"in {len(idle)} gaps, {len(seg)} kernels")


if __name__ == "__main__":
    main()
