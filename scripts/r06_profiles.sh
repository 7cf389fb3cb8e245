# Round-6 evidence on the current tree: rocprofv3 summaries of the headline (pipelined and serial)
# and of every config line's kernels, then every config line at its stated size (which reads those
# summaries for its physical fractions) -> gpurun_out/prof_<tag>/ (summarised into profiles/ on the
# host) and gpurun_out/r06_configs_final.jsonl.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-ceilings"
bash scripts/prof.sh r06_headline trace,fetch,write,sq,mix -- $B || exit $?
SERIAL=1 bash scripts/prof.sh r06_serial trace,sq,mix -- $B || exit $?
bash scripts/prof.sh r06_c5 trace,fetch,write,sq,mix -- bench_configs.py --only C5 || exit $?
bash scripts/prof.sh r06_c5c trace,fetch,sq,mix,tcp,lds -- bench_configs.py --only C5c || exit $?
bash scripts/prof.sh r06_c5f trace,sq,mix -- bench_configs.py --only C5f || exit $?
bash scripts/prof.sh r06_c5e trace,fetch,write,sq,mix -- bench_configs.py --only C5e || exit $?
bash scripts/prof.sh r06_hs trace,sq,mix -- bench_configs.py --only HS || exit $?
bash scripts/prof_configs.sh r06 C2,C3,C4,VG,SG,S || exit $?
cp profiles/r06_*_summary.json gpurun_out/ 2>/dev/null
timeout -k 10 1500 python -u bench_configs.py > gpurun_out/r06_configs_final.jsonl 2> gpurun_out/r06_configs_final.err
rc=$?; echo "configs rc=$rc"; cut -c1-160 gpurun_out/r06_configs_final.jsonl; exit $rc
