# Round 3 final evidence, part C: rocprofv3 kernel stats + PMC passes of the grid and R-stream lines.
set -o pipefail
for c in VG SG C2 C3 C5c R1; do
  t=$(echo $c | tr 'A-Z' 'a-z')
  TAG=r03_$t bash scripts/gpu_prof_cfg.sh python3 bench_configs.py --only $c --c3-reps 512 || exit $?
done
echo all-profiled
