# GPU session: lane-walk step/budget sweep (lower budgets) on config 5 and 20k spheres.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
VARIANTS="s3b8 s3b12 s3b16 s4b10 s4b12 s6b8 s8b6" CONFIGS="c5 s20k" ROUNDS=3 bash tools/gpu_ab.sh > gpurun_out/ab7.log 2>&1 || exit $?
exit 0
