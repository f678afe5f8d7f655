"""Wall vs busy time of a rocprofv3 kernel-trace db over its last N seconds of kernels, plus the
kernel-time share by kernel family (the first word of the demangled name).

usage: python tools/busy.py DB [--last-ms 400]
"""
import argparse
import collections
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-ms", type=float, default=0, help="only kernels in the trailing window")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = list(con.execute("select name, start, end from kernels order by start"))
    if a.last_ms > 0:
        t_end = max(r[2] for r in rows)
        rows = [r for r in rows if r[1] >= t_end - a.last_ms * 1e6]
    busy, cur_s, cur_e = 0, None, None
    for _, s, e in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = rows[-1][2] - rows[0][1]
    fam = collections.Counter()
    cnt = collections.Counter()
    for n, s, e in rows:
        k = re.sub(r"\(anonymous namespace\)::", "", n)
        k = re.split(r"[<(]", k)[0].strip().split(" ")[-1]
        fam[k] += e - s
        cnt[k] += 1
    tot = sum(fam.values())
    print(f"kernels {len(rows)}  wall {wall / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  "
          f"({100 * busy / wall:.1f}%)  kernel-time {tot / 1e6:.2f} ms")
    # idle gaps between consecutive kernels (a start after every earlier kernel's end)
    edges = [0, 2, 5, 10, 20, 50, 200, 1e12]
    gc, gs = [0] * (len(edges) - 1), [0.0] * (len(edges) - 1)
    last_e = rows[0][2]
    for _, s, e in rows[1:]:
        if s > last_e:
            g = (s - last_e) / 1e3
            i = next(j for j in range(len(edges) - 1) if g < edges[j + 1])
            gc[i] += 1
            gs[i] += g
        last_e = max(last_e, e)
    print("idle gaps (us bins): " + "  ".join(
        f"[{edges[i]:g},{edges[i + 1]:g}) n={gc[i]} {gs[i] / 1e3:.2f}ms" for i in range(len(gc))
        if gc[i]).replace("1e+12", "inf"))
    for k, v in fam.most_common(40):
        print(f"{v / 1e6:10.3f} ms {100 * v / tot:6.2f}% {cnt[k]:7d}  {k[:90]}")


if __name__ == "__main__":
    main()
