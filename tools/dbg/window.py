"""Print every kernel in a time window of a rocprofv3 kernel-trace db: start, duration, queue.
usage: python tools/dbg/window.py DB ANCHOR_SUBSTR INDEX WINDOW_US"""
import re
import sqlite3
import sys

db, anchor, idx, win = sys.argv[1], sys.argv[2], int(sys.argv[3]), float(sys.argv[4])
con = sqlite3.connect(db)
rows = list(con.execute("select name, start, end, queue_id from kernels order by start"))
anc = [r for r in rows if anchor in r[0]]
t0 = anc[idx][1]
busy_end, busy = t0, 0
for name, s, e, q in rows:
    if s < t0 or s > t0 + win * 1e3:
        continue
    n = re.sub(r"\(.*", "", re.sub(r"\(anonymous namespace\)::", "", name))[:50]
    print(f"{(s - t0) / 1e3:8.2f}  dur {(e - s) / 1e3:7.2f}  q{q}  {n}")
    if e > busy_end:
        busy += e - max(s, busy_end)
        busy_end = e
print(f"busy {busy / 1e3:.1f} us of {win} us")
