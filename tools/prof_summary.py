"""Summarise a rocprofv3 results db: top kernels, per-forward time. usage: prof_summary.py DB [n_fwd]"""
import re
import sqlite3
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"at::native::", "", n)
    return n[:110]


def main():
    db = sys.argv[1]
    nfwd = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    con = sqlite3.connect(db)
    rows = list(con.execute("select name,total_calls,total_duration,average,percentage from top_kernels"))
    tot = sum(r[2] for r in rows)
    print(f"total kernel time {tot/1e3:.2f} ms, per forward {tot/1e3/nfwd:.3f} ms ({nfwd} fwd)")
    for n, c, t, a, p in rows[:25]:
        print(f"{p:6.2f}%  {t/nfwd:9.1f} us/fwd  {c/nfwd:6.1f} calls/fwd  avg {a:8.2f} us  {short(n)}")


if __name__ == "__main__":
    main()
