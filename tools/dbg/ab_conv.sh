# A/B the conv variants in scflow_amd/lib/ab/*.so on chosen shapes: tools/dbg/ab_conv.sh "shapes" batch variant...
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab; mkdir -p $O
SH=$1; B=$2; shift 2
timeout -k 10 120 python tools/conv_bench.py --batch $B --only "$SH" --no-extras > $O/base.txt 2>&1 || exit 1
for v in "$@"; do
  SCFLOW_LIB=$R/scflow_amd/lib/ab/$v.so timeout -k 10 120 python tools/conv_bench.py --batch $B --only "$SH" --no-extras > $O/$v.txt 2>&1 || exit 2
done
