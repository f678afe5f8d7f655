"""Average PMC counters per kernel (grouped by name + grid) from rocprofv3 csv output."""
import csv
import collections
import re
import sys


def load(path):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])[:60]
        key = (name, r.get("Grid_Size", r.get("Grid_Size_X", "")), r.get("Workgroup_Size", ""))
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


if __name__ == "__main__":
    for path in sys.argv[1:]:
        print("==", path)
        agg = load(path)
        for key, ctrs in sorted(agg.items()):
            vals = {c: sum(v) / len(v) for c, v in ctrs.items()}
            print(key, {c: f"{v:.4g}" for c, v in sorted(vals.items())})
