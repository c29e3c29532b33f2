# GPU session: drop-in variants at the shipped tc = 4 (pinned g_data vs copy-back,
# batching off), then A/B of $VARIANTS on $CONFIGS.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
H=simplepathtracer_amd/lib/spt_dropin_harness
: > gpurun_out/dropin_var.log
for env in "SPT_PIN=1" "SPT_PIN=0" "SPT_BATCH=0" "SPT_PIN=1" "SPT_PIN=0"; do
  for t in 0 1; do
    echo "$env task=$t $(env $env timeout -k 10 120 $H /dev/null 1200 800 100 50 4 $t 5)" >> gpurun_out/dropin_var.log || exit $?
  done
done
VARIANTS="$VARIANTS" CONFIGS="${CONFIGS:-c2}" bash tools/gpu_ab.sh > gpurun_out/ab.log 2>&1 || exit $?
exit 0
