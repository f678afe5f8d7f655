"""Write a rocprofv3 run db's top_kernels table as a text summary (profiles/*.txt).

usage: python tools/stats_file.py DB "command line" > profiles/NAME.txt
"""
import re
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
print(f"rocprofv3 --kernel-trace --stats -- {sys.argv[2] if len(sys.argv) > 2 else ''}")
print(f"{'calls':>7} {'total_ms':>10} {'avg_us':>10} {'pct':>6}  kernel")
for n, c, t, a, p in con.execute("select name,total_calls,total_duration,average,percentage from top_kernels"):
    n = re.sub(r"\(anonymous namespace\)::", "", n)[:110]
    print(f"{c:7d} {t / 1e3:10.2f} {a:10.2f} {p:6.2f}  {n}")
