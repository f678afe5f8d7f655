"""How far the host runs ahead of the GPU, per kernel of one decoder iteration, from a rocprofv3
``--kernel-trace --hip-trace`` db: for each kernel, the end of the HIP API call that enqueued it
(joined on the correlation id) relative to the kernel's start.  A negative lead means the GPU
reached that point of the queue before the host had written the launch: the gap in front of the
kernel is host time, not device time.

usage: python tools/host_lead.py DB [--iteration I] [--marker NAME]
"""
import argparse
import re
import sqlite3


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*", "", n)
    return n[:56]


def cols(con, view):
    try:
        return [r[1] for r in con.execute(f"pragma table_info({view})")]
    except sqlite3.Error:
        return []


def pick(names, *cands):
    for c in cands:
        if c in names:
            return c
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--iteration", type=int, default=60)
    ap.add_argument("--marker", default="corr_lookup")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    views = [r[0] for r in con.execute("select name from sqlite_master where type in ('view','table')")]
    kc = cols(con, "kernels")
    rview = pick(views, "regions", "hip_api", "region")
    rc = cols(con, rview) if rview else []
    kcorr = pick(kc, "correlation_id", "corr_id", "stack_id")
    rcorr = pick(rc, "correlation_id", "corr_id", "stack_id")
    if not (kcorr and rcorr):
        print("views:", views)
        print("kernels:", kc)
        print(rview, rc)
        return
    api = {}
    for cid, name, s, e in con.execute(f"select {rcorr}, name, start, end from {rview}"):
        api[cid] = (name, s, e)
    rows = list(con.execute(f"select name, start, end, queue_id, {kcorr} from kernels order by start"))
    starts = [i for i, r in enumerate(rows) if a.marker in r[0]]
    lo, hi = starts[a.iteration], starts[a.iteration + 1]
    seg = rows[lo:hi]
    t0 = seg[0][1]
    print(f"{'start':>9}  {'dur':>6}  q  {'lead':>8}  kernel  (lead = kernel start - end of its launch call)")
    for name, s, e, q, cid in seg:
        lead = ""
        if cid in api:
            lead = f"{(s - api[cid][2]) / 1e3:8.1f}"
        print(f"{(s - t0) / 1e3:9.2f}  {(e - s) / 1e3:6.2f}  q{q}  {lead:>8}  {short(name)}")
    # the host's API calls between the iteration's first and last kernel start
    calls = [(s, e, n) for (n, s, e) in api.values() if t0 - 2_000_000 <= s <= seg[-1][1]]
    print(f"{len(calls)} HIP API calls in the window")


if __name__ == "__main__":
    main()
