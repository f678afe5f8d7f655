#!/bin/bash
# Round 5, session T: at configs[1], the fused lookup + corr_net.0 vs the separate tile-row lookup
# (two level regions per slot, round 5) + the wide 1×1 conv, vs the separate tile-region lookup;
# then the PMC passes for the configs[4] F(2×2,3×3) traffic group.
set -o pipefail
O=gpurun_out/r5t; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_bench.py --rounds 5 --steps 10 fuse_lookup_conv=1,0 > $O/ab_fuse_tr.txt 2>&1 || exit 2
SCFLOW_LK_TILEREG=0 timeout -k 10 300 python -u tools/ab_bench.py --rounds 5 --steps 10 fuse_lookup_conv=1,0 > $O/ab_fuse_tb.txt 2>&1 || exit 3
SCFLOW_LK_TILEREG=0 timeout -k 10 120 python -u tools/lookup_bench.py --reps 50 --stamps --batch 16 --size 256 2>&1 | grep -v amdgpu.ids | sed "s/^/tb /" >> $O/lookup_c1.txt || exit 4
timeout -k 10 120 python -u tools/lookup_bench.py --reps 50 --stamps --batch 16 --size 256 2>&1 | grep -v amdgpu.ids | sed "s/^/tr /" >> $O/lookup_c1.txt || exit 4
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_r5t; mkdir -p $OUT
cd /tmp
P="--steps 2 --warmup 1 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --no-kernel-timer --batch 32 --size 512 --iters 12"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_c4 -o run -- python3 $R/bench.py $P > /dev/null 2> $OUT/f.err || exit 5
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_c4 -o run -- python3 $R/bench.py $P > /dev/null 2> $OUT/w.err || exit 5
python3 $R/tools/traffic_json.py $OUT/fetch_c4 $OUT/write_c4 --batch 32 --size 512 --iters 12 > $OUT/traffic_b32_s512.json
rm -rf $OUT/fetch_c4 $OUT/write_c4
