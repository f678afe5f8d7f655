#!/bin/bash
# Round 5, session B: the tile-row lookup regions (SCFLOW_LK_TB) — parity, standalone A/B with
# phase stamps and PMC passes at configs[4]; configs[4] decoder A/B; training-switch A/B, one
# switch at a time on the static-wgrad library.
set -o pipefail
O=gpurun_out/r5b; mkdir -p $O; export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -rfs --timeout 120 --timeout-method thread -k "tiled or lookup" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for tb in 0 1; do
    SCFLOW_LK_TB=$tb timeout -k 10 120 python -u tools/lookup_bench.py --reps 50 --stamps $([ $rep = 1 ] && echo --check) 2>&1 | grep -v amdgpu.ids | sed "s/^/tb$tb /" >> $O/lookup.txt || exit 3
  done
done
for tb in 0 1; do
  SCFLOW_LK_TB=$tb timeout -k 10 120 python -u tools/lookup_bench.py --reps 50 --stamps --flow-scale 1 2>&1 | grep -v amdgpu.ids | sed "s/^/tb$tb flow1 /" >> $O/lookup.txt || exit 3
done
cd /tmp
for tb in 0 1; do
  SCFLOW_LK_TB=$tb timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$tb -o run -- python3 $R/tools/lookup_bench.py --reps 5 > /dev/null 2> $R/$O/f$tb.err || exit 4
  SCFLOW_LK_TB=$tb timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w$tb -o run -- python3 $R/tools/lookup_bench.py --reps 5 > /dev/null 2> $R/$O/w$tb.err || exit 4
  SCFLOW_LK_TB=$tb timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/s$tb -o run -- python3 $R/tools/lookup_bench.py --reps 5 > /dev/null 2> $R/$O/s$tb.err || exit 4
  python3 $R/tools/pmc_summary.py $(find $R/$O/f$tb $R/$O/w$tb $R/$O/s$tb -name "*counter_collection.csv") | grep -i lookup | cut -c1-900 > $R/$O/pmc_tb$tb.txt
  rm -rf $R/$O/f$tb $R/$O/w$tb $R/$O/s$tb
done
cd $R
B="--steps 5 --warmup 2 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --batch 32 --size 512 --iters 12"
for rep in 1 2; do
  for tb in 0 1; do
    SCFLOW_LK_TB=$tb timeout -k 10 200 python -u bench.py $B > $O/c4_tb${tb}_$rep.json 2> $O/c4_tb${tb}_$rep.err || exit 5
  done
done
WS=scflow_amd/lib/ab/ws1.so
for rep in 1 2; do
  for v in base BN RELU HEADS RES; do
    E=""; [ $v != base ] && E="SCFLOW_TRAIN_${v}_FUSED=1"
    [ $v = RELU ] && E="SCFLOW_TRAIN_RELU_MASK=1"
    [ $v = RES ] && E="SCFLOW_TRAIN_RES_GRAD=1"
    env $E SCFLOW_LIB=$WS timeout -k 10 300 python -u tools/train_timing.py --steps 12 --freeze > $O/tt_${v}_$rep.json 2> $O/tt_${v}_$rep.err || exit 6
    echo "$v $rep $(head -c 300 $O/tt_${v}_$rep.json)" >> $O/tt.txt
  done
done
