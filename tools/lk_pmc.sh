R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/pmc_lk; mkdir -p $OUT; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python3 $R/tools/conv_bench.py --reps 2 > $OUT/p1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $OUT/p2 -o run -- python3 $R/tools/conv_bench.py --reps 2 > $OUT/p2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p3 -o run -- python3 $R/tools/conv_bench.py --reps 2 > $OUT/p3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p4 -o run -- python3 $R/tools/conv_bench.py --reps 2 > $OUT/p4.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py $(find $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 -name "*counter_collection.csv") | grep -i "lookup" | cut -c1-900
