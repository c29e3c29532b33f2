# GPU session: lane-walk step variants on config 5 (A/B), drop-in batch shape sweep at
# tc = 4, device-path block/grid knobs on config 2.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
VARIANTS="s2 s2b28 s3" CONFIGS=c5 bash tools/gpu_ab.sh > gpurun_out/ab5.log 2>&1 || exit $?
H=simplepathtracer_amd/lib/spt_dropin_harness
: > gpurun_out/dropin_sweep.log
for env in "SPT_BATCH_SETS=2" "SPT_BATCH_SETS=2 SPT_BATCH_GRID_DIV=2" "SPT_BATCH_SETS=3 SPT_BATCH_GRID_DIV=2" \
           "SPT_BATCH_SETS=4 SPT_BATCH_GRID_DIV=2" "SPT_BATCH_SETS=4 SPT_BATCH_GRID_DIV=3" "SPT_BATCH_SETS=2"; do
  echo "$env $(env $env timeout -k 10 120 $H /dev/null 1200 800 100 50 4 0 8)" >> gpurun_out/dropin_sweep.log || exit $?
done
: > gpurun_out/grid_sweep.log
for env in "SPT_X=0" "SPT_BLOCKS_PER_CU=7" "SPT_BLOCKS_PER_CU=6" "SPT_X=0"; do
  echo "$env $(env $env timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin | tail -1 | cut -c1-330)" >> gpurun_out/grid_sweep.log || exit $?
done
exit 0
