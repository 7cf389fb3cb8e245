# Round-2 final measurement call: the default bench line, the headline rocprofv3 passes (serial
# chunks and the two-stream pipeline), every config line, and the C5 / C5-continuous kernel
# traces.  Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for MODE in ser hl; do
  if [ $MODE = ser ]; then export DCOR_SIGN_PIPELINE=0; else export DCOR_SIGN_PIPELINE=1; fi
  D=$O/$MODE
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_trace -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $D/trace.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/prof_fetch -o run -- $B > $D/fetch.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/prof_write -o run -- $B > $D/write.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $D/prof_sq -o run -- $B > $D/sq.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU --output-format csv -d $D/prof_mix -o run -- $B > $D/mix.log 2>&1 || exit $?
  echo "profile $MODE done"
done
unset DCOR_SIGN_PIPELINE
timeout -k 10 900 python -u bench_configs.py > $O/configs.jsonl 2> $O/configs.err || exit $?
echo "configs done"
for C in C5 C5c; do
  D=$O/c5t/$C
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_trace -o run -- python3 bench_configs.py --only $C > $D/trace.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/prof_fetch -o run -- python3 bench_configs.py --only $C > $D/fetch.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $D/prof_sq -o run -- python3 bench_configs.py --only $C > $D/sq.log 2>&1 || exit $?
done
echo "c5 traces done"
