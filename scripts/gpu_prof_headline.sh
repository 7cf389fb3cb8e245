# Headline rocprofv3 passes (kernel trace + PMC): TAG=r01_headline bash scripts/gpu_prof_headline.sh
# PIPE=0 profiles the chunks serially (clean per-kernel counters).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
export DCOR_SIGN_PIPELINE=${PIPE:-1}
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- $B > $O/prof_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- $B > $O/prof_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/prof_sq -o run -- $B > $O/prof_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU --output-format csv -d $O/prof_mix -o run -- $B > $O/prof_mix.log 2>&1 || exit $?
echo done
