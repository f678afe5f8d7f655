#!/bin/bash
# Round 5, session I: the whole GPU suite at the current tree, then A/Bs of this round's later
# changes, library by library (SCFLOW_LIB):
#   old  = HEAD before them (Winograd halo pitches)
#   mid  = + 16-B typed thin-conv halos, conflict-free enc_conv A halos, tap-extent loads in the
#          fused lookup + corr_net.0
#   new  = + the GRU epilogue's global reads issued before its LDS exchange
#   tb2  = + the tile-row lookup with two level regions per pixel slot (6 workgroups per CU)
set -o pipefail
O=gpurun_out/r5i; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rfs -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in old mid new tb2; do
    SCFLOW_LIB=scflow_amd/lib/ab/$v.so timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || exit 3
  done
done
for rep in 1 2; do
  for v in new tb2; do
    SCFLOW_LIB=scflow_amd/lib/ab/$v.so timeout -k 10 120 python -u tools/lookup_bench.py --reps 50 --stamps $([ $rep = 1 ] && echo --check) 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" >> $O/lookup.txt || exit 4
  done
done
for v in old tb2; do
  SCFLOW_LIB=scflow_amd/lib/ab/$v.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12 > $O/bench_c4_$v.json 2> $O/bench_c4_$v.err || exit 5
done
timeout -k 10 400 python -u tools/ab_bench.py --batch 32 --size 512 --iters 12 --rounds 3 --steps 4 fuse_lookup_conv_max_px=1024,4096 > $O/ab_c4_fuse.txt 2>&1 || exit 6
for v in mid new; do
  SCFLOW_LIB=scflow_amd/lib/ab/$v.so timeout -k 10 150 python -u tools/conv_bench.py --no-extras --reps 20 --stamps --xcd --only "gru" 2>&1 | grep -v amdgpu | sed "s/^/$v /" >> $O/stamps.txt || exit 7
done
