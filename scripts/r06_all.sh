# Round-6 final: the driver's gate (every -m gpu test, smoke), bench.py with its defaults, then the
# rocprofv3 evidence and every config line (scripts/r06_profiles.sh).
set -o pipefail
export TMPDIR=/tmp
bash scripts/r06_final.sh || exit $?
bash scripts/r06_profiles.sh
