# Serial-chunk kernel trace + VALU counters of the headline (per-kernel times of pass 1 / pass 2 / epilogue).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ser}
mkdir -p $O
export DCOR_SIGN_PIPELINE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_trace.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/prof_sq -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_sq.log 2>&1 || exit $?
f=$(find $O/prof_trace -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -8
