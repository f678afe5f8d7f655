set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu $R/tests/test_gpu_encoder.py $R/tests/test_gpu_configs.py $R/tests/test_gpu_train.py > $OUT/stem_tests.log 2>&1 || { tail -30 $OUT/stem_tests.log; exit 1; }
tail -2 $OUT/stem_tests.log
timeout -k 10 300 python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/stem_bench.json 2> $OUT/stem_bench.err || exit $?
SCFLOW_STEM_MFMA=0 timeout -k 10 300 python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/stem_bench_valu.json 2>> $OUT/stem_bench.err || exit $?
python -c "
import json,sys
for f in ['stem_bench_valu.json','stem_bench.json']:
    d=json.loads(open('$OUT/'+f).read().strip().splitlines()[-1]); print(f, d['value'], d['end_to_end']['value'], d['end_to_end']['ms_per_step'], d['training_step']['ms_per_step'])
"
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/stemprof -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 3 --train-batch 0 > /dev/null 2> $OUT/stemprof.err || exit $?
DB=$(find $OUT/stemprof -name "*.db" | head -1)
python3 $R/tools/stats_file.py $DB "python bench.py --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 3 --train-batch 0" > $OUT/stem_e2e_stats.txt
rm -rf $OUT/stemprof
head -25 $OUT/stem_e2e_stats.txt
