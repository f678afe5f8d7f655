#!/bin/bash
# One GPU-box session, as a list of named steps (replaces the round-4/5 one-off sess_*.sh).
# Every step runs under its own time limit; the session stops at the first step that fails
# (pytest exit 1 included), so nothing more touches the GPU after a fault, abort or time-out.
#
# usage: tools/session.sh TAG STEP [STEP ...]        → gpurun_out/s_TAG/
#   test                 whole GPU suite, no -x (every collected test reached)
#   test=EXPR            GPU tests matching -k EXPR, -x
#   smoke                __graft_entry__.smoke()
#   bench[=ARGS]         bench.py [ARGS]                      → bench.json
#   c4                   configs[4] bench line (B=32, 512², 12 iterations) → bench_c4.json
#   dec[=ARGS]           decoder-only bench leg, 20 steps     → dec.json (one line printed)
#   conv=B:S:ONLY[:stamps]   tools/conv_bench.py at batch B, feature size S, shapes ONLY
#   ab=NAME:B:S:ONLY     variant scflow_amd/lib/ab/NAME.so (tools/build_variant.sh) vs the default
#                        library: conv_bench ONLY at B×S² and the decoder at that config, 2 rounds
#   abenv=VAR:V1,V2:B:S:ONLY   the same A/B over the values of an environment switch
#   abdec=TOGGLES        tools/ab_bench.py TOGGLES (';' separates arguments)
#   quick[=ARGS]         kernel trace of the decoder leg: per-forward table + iteration timeline
#   traffic=NAME:c1|c4[:VAR=VAL]   FETCH_SIZE + WRITE_SIZE passes (each its own rocprofv3 run)
#                        over the decoder leg → traffic_NAME.json (tools/traffic_json.py)
#   pmc=NAME;LIB;CTRS;SCRIPT[;ARGS…]   one rocprofv3 --pmc pass (CTRS space-separated, within one
#                        pass's limits) over python tools/SCRIPT ARGS with scflow_amd/lib/ab/LIB.so
#                        (LIB = base: the default library) → pmc_NAME.txt (tools/pmc_summary.py)
#   pyab=LIB;SCRIPT[;ARGS…]   python tools/SCRIPT ARGS with the default library and with
#                        scflow_amd/lib/ab/LIB.so, alternating, 2 rounds
#   trainprof[=ENV]      kernel trace of 5 training steps (tools/train_bench.py) → train_stats.txt
#   prof                 tools/prof_r5.sh TAG (HEAD evidence: traces, timeline, PMC, traffic)
#   py=SCRIPT[;ARGS]     python tools/SCRIPT ARGS ('; ' separates arguments)
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/s_$TAG; mkdir -p $OUT; cd $R; export TMPDIR=/tmp
DEC="--no-cpu-baseline --e2e-batch 0 --train-batch 0"
C4="--batch 32 --size 512 --iters 12"
line() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['value'], d['ms_per_step'], d.get('roofline',{}).get('frac'))" "$@"; }
cfg() { [ "$2" = 64 ] && echo "$C4" || echo "--batch $1"; }  # conv_bench size → bench config

for STEP in "$@"; do
  K=${STEP%%=*}; V=${STEP#*=}; [ "$V" = "$STEP" ] && V=""
  echo "== $STEP"
  case $K in
    test)
      if [ -z "$V" ]; then
        timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
      else
        timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread -p no:cacheprovider -k "$V" > $OUT/gputest.log 2>&1
      fi
      rc=$?; tail -3 $OUT/gputest.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit 5
      tail -2 $OUT/smoke.txt ;;
    bench)
      timeout -k 10 500 python bench.py $V > $OUT/bench.json 2> $OUT/bench.err || exit 6
      line $OUT/bench.json bench ;;
    c4)
      timeout -k 10 300 python bench.py $C4 --no-cpu-baseline --e2e-batch 0 --train-batch 0 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 7
      line $OUT/bench_c4.json c4 ;;
    dec)
      timeout -k 10 300 python bench.py --steps 20 --warmup 3 $DEC $V > $OUT/dec.json 2> $OUT/dec.err || exit 8
      line $OUT/dec.json dec ;;
    conv)
      IFS=: read B S ONLY ST <<< "$V"
      timeout -k 10 300 python tools/conv_bench.py --batch $B --size $S --only "$ONLY" --no-extras --reps 50 ${ST:+--stamps} 2>&1 | grep -v amdgpu.ids | tee -a $OUT/conv.txt
      [ ${PIPESTATUS[0]} -eq 0 ] || exit 9 ;;
    ab|abenv)
      if [ $K = ab ]; then
        IFS=: read NAME B S ONLY <<< "$V"; LIB=$R/scflow_amd/lib/ab/$NAME.so
        [ -f $LIB ] || { echo "missing $LIB"; exit 2; }; VARS="base $NAME"
      else
        IFS=: read VAR VALS B S ONLY <<< "$V"; VARS=${VALS//,/ }
      fi
      for r in 1 2; do
        for v in $VARS; do
          if [ $K = ab ]; then E="SCFLOW_LIB="; [ $v != base ] && E="SCFLOW_LIB=$LIB"; else E="$VAR=$v"; fi
          env $E timeout -k 10 200 python tools/conv_bench.py --batch $B --size $S --only "$ONLY" --no-extras --reps 50 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" | tee -a $OUT/ab.txt
          [ ${PIPESTATUS[0]} -eq 0 ] || exit 10
          env $E timeout -k 10 300 python bench.py --steps 12 --warmup 3 $DEC $(cfg $B $S) > $OUT/ab_$v$r.json 2> $OUT/ab_$v$r.err || exit 10
          line $OUT/ab_$v$r.json "$v dec" | tee -a $OUT/ab.txt
        done
      done ;;
    abdec)
      IFS=';' read -ra A <<< "$V"
      timeout -k 10 600 python tools/ab_bench.py "${A[@]}" 2>&1 | grep -v amdgpu.ids | tee -a $OUT/abdec.txt
      [ ${PIPESTATUS[0]} -eq 0 ] || exit 11 ;;
    quick)
      cd /tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 $DEC $V > /dev/null 2> $OUT/kt.err || exit 12
      DB=$(find $OUT/kt -name "*.db" | head -1)
      python3 $R/tools/prof_summary.py $DB 24 > $OUT/per_forward.txt
      python3 $R/tools/timeline.py $DB --iteration 61 > $OUT/timeline.txt 2>&1
      rm -rf $OUT/kt; cd $R
      head -20 $OUT/per_forward.txt; tail -1 $OUT/timeline.txt ;;
    traffic)
      IFS=: read NAME CF EV <<< "$V"
      P="--steps 2 --warmup 1 --no-cpu-baseline --e2e-batch 0 --train-batch 0 --no-kernel-timer"
      TJ="--batch 16 --size 256 --iters 8"
      [ "$CF" = c4 ] && { P="$P $C4"; TJ="--batch 32 --size 512 --iters 12"; }
      cd /tmp
      for ctr in FETCH_SIZE WRITE_SIZE; do
        env $EV timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_${NAME}_$ctr -o run -- python3 $R/bench.py $P > /dev/null 2> $OUT/pmc_${NAME}_$ctr.err || exit 15
      done
      cd $R
      python3 tools/traffic_json.py $OUT/pmc_${NAME}_FETCH_SIZE $OUT/pmc_${NAME}_WRITE_SIZE $TJ > $OUT/traffic_$NAME.json || exit 15
      rm -rf $OUT/pmc_${NAME}_*
      python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))
for k,v in d['kernels'].items():
    print(f\"{k:28s} {v['hbm_bytes_per_launch']/1e6:9.1f} MB/launch  x{v['ratio_to_algorithmic']}\")" $OUT/traffic_$NAME.json ;;
    pmc)
      IFS=';' read -ra A <<< "$V"
      NAME=${A[0]}; LIB=${A[1]}; CTRS=${A[2]}; SCR=${A[3]}
      E="SCFLOW_LIB="; [ "$LIB" != base ] && E="SCFLOW_LIB=$R/scflow_amd/lib/ab/$LIB.so"
      cd /tmp
      env $E timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/pmc_$NAME -o run -- python3 $R/tools/$SCR "${A[@]:4}" > $OUT/pmc_$NAME.log 2>&1 || exit 16
      cd $R
      python3 tools/pmc_summary.py $(find $OUT/pmc_$NAME -name "*counter_collection.csv") > $OUT/pmc_$NAME.txt
      rm -rf $OUT/pmc_$NAME
      grep -v "^==" $OUT/pmc_$NAME.txt | sed "s/^/$NAME /" | cut -c1-400 ;;
    pyab)
      IFS=';' read -ra A <<< "$V"
      LIB=$R/scflow_amd/lib/ab/${A[0]}.so; [ -f $LIB ] || { echo "missing $LIB"; exit 2; }
      for r in 1 2; do
        for v in base ${A[0]}; do
          E="SCFLOW_LIB="; [ $v != base ] && E="SCFLOW_LIB=$LIB"
          env $E timeout -k 10 300 python tools/"${A[@]:1}" 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" | tee -a $OUT/pyab.txt
          [ ${PIPESTATUS[0]} -eq 0 ] || exit 18
        done
      done ;;
    trainprof)
      cd /tmp
      env $V timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/ktt -o run -- python3 $R/tools/train_bench.py --steps 3 --warmup 2 > $OUT/train_bench.json 2> $OUT/ktt.err || exit 17
      DB=$(find $OUT/ktt -name "*.db" | head -1)
      python3 $R/tools/stats_file.py $DB "python tools/train_bench.py --steps 3 --warmup 2 (5 training steps, B=16, 256x256, 8 iters)" > $OUT/train_stats.txt
      rm -rf $OUT/ktt; cd $R
      head -30 $OUT/train_stats.txt ;;
    prof)
      bash tools/prof_r5.sh $TAG || exit 13 ;;
    py)
      IFS=';' read -ra A <<< "$V"
      timeout -k 10 400 python tools/"${A[@]}" 2>&1 | grep -v amdgpu.ids | tee -a $OUT/py.txt
      [ ${PIPESTATUS[0]} -eq 0 ] || exit 14 ;;
    *) echo "unknown step $K"; exit 2 ;;
  esac
done
