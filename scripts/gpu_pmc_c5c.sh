# C5 / C5-continuous PMC passes (kernel trace, FETCH_SIZE, WRITE_SIZE, SQ activity, LDS) for
# the coded kernel, the tiled kernel and the L2-gather kernel: gpurun_out/c5p/{coded,tiled,l2}.
set -o pipefail
export TMPDIR=/tmp
for MODE in coded tiled l2; do
  D=gpurun_out/c5p/$MODE
  mkdir -p $D
  unset DCOR_TILED
  C=C5c
  if [ $MODE = coded ]; then C=C5; fi
  if [ $MODE = l2 ]; then export DCOR_TILED=0; fi
  B="python3 bench_configs.py --only $C"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_trace -o run -- $B > $D/trace.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/prof_fetch -o run -- $B > $D/fetch.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/prof_write -o run -- $B > $D/write.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $D/prof_sq -o run -- $B > $D/sq.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --output-format csv -d $D/prof_mix -o run -- $B > $D/mix.log 2>&1 || exit $?
  echo "$MODE done"
done
