# GPU session: leaf-pass threshold sweep on the 6-step lane walk; drop-in tc = 4 / 32
# with the batch grid halved.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
VARIANTS="t32 t24 t16 t32b10 t24b10 t32s4" CONFIGS="c5 s20k" ROUNDS=3 bash tools/gpu_ab.sh > gpurun_out/ab9.log 2>&1 || exit $?
H=simplepathtracer_amd/lib/spt_dropin_harness
: > gpurun_out/dropin_div.log
for env in "SPT_BATCH_GRID_DIV=1" "SPT_BATCH_GRID_DIV=2" "SPT_BATCH_GRID_DIV=1" "SPT_BATCH_GRID_DIV=2"; do
  for tc in 4 32; do
    echo "$env tc=$tc $(env $env timeout -k 10 120 $H /dev/null 1200 800 100 50 $tc 0 8)" >> gpurun_out/dropin_div.log || exit $?
  done
done
exit 0
