# rocprofv3 recipe for any workload: a kernel trace, then PMC passes (each in its own run, as the
# guide prescribes), then profiles/<tag>_summary.{json,md} + <tag>_kernel_stats.csv.
#   bash scripts/prof.sh <tag> <passes> -- <python args...>
# passes: comma list of trace, fetch, write, sq, mix, tcp, lds (default trace,fetch,write,sq,mix)
# env: SERIAL=1 runs the sign path's chunks on one stream (--variant DCOR_SIGN_PIPELINE=0: clean per-kernel
#      counters); PROF_HEAD=<git head> is stamped into the summary (the GPU box has no .git).
# Example: bash scripts/prof.sh r04_serial trace,sq,mix -- bench.py --steps 5 --warmup 1 --no-cpu-baseline
set -o pipefail
export TMPDIR=/tmp
TAG=$1; PASSES=${2:-trace,fetch,write,sq,mix}; shift 2
[ "$1" = "--" ] && shift
O=gpurun_out/prof_$TAG
rm -rf $O; mkdir -p $O
EXTRA=()
[ "${SERIAL:-0}" = 1 ] && EXTRA=(--variant DCOR_SIGN_PIPELINE=0)
export PROF_CMD="SERIAL=${SERIAL:-0} bash scripts/prof.sh $TAG $PASSES -- $*"
pmc() {  # one PMC pass: name, counters...
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $O/prof_$n -o run -- python3 "${ARGS[@]}" > $O/prof_$n.log 2>&1
}
ARGS=("$@" "${EXTRA[@]}")
for p in ${PASSES//,/ }; do
  case $p in
    trace) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o run -- python3 "${ARGS[@]}" > $O/prof_trace.log 2>&1 ;;
    fetch) pmc fetch FETCH_SIZE ;;
    write) pmc write WRITE_SIZE ;;
    sq) pmc sq SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE ;;
    mix) pmc mix SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU ;;
    lds) pmc lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE ;;
    tcp) pmc tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE ;;
    *) echo "unknown pass $p"; exit 2 ;;
  esac
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $p rc=$rc"; tail -5 $O/prof_$p.log; exit $rc; fi
done
python3 scripts/summarize_prof.py $TAG $O && echo "profiles/${TAG}_summary.json"
