cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/e2e_prof -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --e2e-steps 3 --train-batch 0 > $R/gpurun_out/e2e_prof.json 2> $R/gpurun_out/e2e_prof.err || exit 1
python3 $R/tools/prof_summary.py $(find $R/gpurun_out/e2e_prof -name "*.db" | head -1) 1 > $R/gpurun_out/e2e_prof.txt
rm -rf $R/gpurun_out/e2e_prof
head -40 $R/gpurun_out/e2e_prof.txt
