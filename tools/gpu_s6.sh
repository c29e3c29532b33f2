# GPU session: lane-walk step/budget sweep on config 5 and a 20k-sphere stress scene
# (global-memory lane walk), drop-in fold placement at tc = 4.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
VARIANTS="s3b16 s3b20 s3b24 s3b32 s4b16 s4b20 s5b14" CONFIGS="c5 s20k" ROUNDS=3 bash tools/gpu_ab.sh > gpurun_out/ab6.log 2>&1 || exit $?
H=simplepathtracer_amd/lib/spt_dropin_harness
: > gpurun_out/dropin_fold.log
for env in "SPT_BATCH_GRID_DIV=2" "SPT_BATCH_GRID_DIV=2 SPT_FOLD_HOST=0" "SPT_FOLD_HOST=0" "SPT_BATCH_GRID_DIV=2"; do
  for t in 0 1; do
    echo "$env task=$t $(env $env timeout -k 10 120 $H /dev/null 1200 800 100 50 4 $t 8)" >> gpurun_out/dropin_fold.log || exit $?
  done
done
exit 0
