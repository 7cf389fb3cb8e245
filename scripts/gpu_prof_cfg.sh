# rocprofv3 passes (kernel trace + the PMC passes scripts/summarize_prof.py reads) over one command:
#   TAG=r03_vg bash scripts/gpu_prof_cfg.sh python3 bench_configs.py --only VG
# -> gpurun_out/$TAG/prof_{trace,fetch,write,sq,mix}; then (here): python scripts/summarize_prof.py $TAG gpurun_out/$TAG
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:?}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o run -- "$@" > $O/prof_trace.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- "$@" > $O/prof_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- "$@" > $O/prof_write.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/prof_sq -o run -- "$@" > $O/prof_sq.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU --output-format csv -d $O/prof_mix -o run -- "$@" > $O/prof_mix.log 2>&1 || exit $?
echo "profiled: $*"
