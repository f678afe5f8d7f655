# The XHead 128→512 Winograd conv under each XCD block order (SCFLOW_WINO_SWZ = column parts
# across the 8 XCDs, 0 = linear): launch time (stamps run) and FETCH_SIZE / WRITE_SIZE per launch
# (separate counter passes), into gpurun_out/heads_swz/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/heads_swz
mkdir -p $OUT
for c in ${SWZ:-0 2 4 8}; do
  SCFLOW_WINO_SWZ=$c timeout -k 10 100 python3 $R/tools/dbg/wino_phases.py --only heads 2>/dev/null \
    | sed "s/^/swz=$c /" | tee -a $OUT/time.txt || exit 1
  for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && SCFLOW_WINO_SWZ=$c timeout -s KILL 90 rocprofv3 --pmc $ctr \
      --output-format csv -d $OUT/p_${c}_$ctr -o run -- python3 $R/tools/dbg/wino_phases.py \
      --only heads --no-stamps > $OUT/p_${c}_$ctr.log 2>&1) || exit 1
    python3 - "$c" "$ctr" $(find $OUT/p_${c}_$ctr -name "*counter_collection.csv") <<'PY' | tee -a $OUT/traffic.txt
import csv, sys
c, ctr, path = sys.argv[1], sys.argv[2], sys.argv[3]
vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
        if "conv_wino_kernel" in r["Kernel_Name"] and r["Counter_Name"] == ctr]
print(f"swz={c} {ctr} launches {len(vals)} avg {sum(vals) / max(1, len(vals)):.0f} KB")
PY
  done
done
