# GPU session: config benches, VALU issue rates, A/B of variants, drop-in batch sets,
# PC sampling (last: beta feature).  Each step bounded; a failed step ends the session.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
bash tools/gpu_cfgs.sh || exit $?
echo cfgs-done
timeout -k 10 60 tools/ubench/issue_rates > gpurun_out/ubench.log 2>&1 || exit $?
echo ubench-done
VARIANTS="$VARIANTS" CONFIGS="${CONFIGS:-c2}" bash tools/gpu_ab.sh > gpurun_out/ab.log 2>&1 || exit $?
echo ab-done
H=simplepathtracer_amd/lib/spt_dropin_harness
for k in 2 3 4; do
  for tc in 4 32; do
    echo "sets=$k tc=$tc $(SPT_BATCH_SETS=$k timeout -k 10 120 $H /dev/null 1200 800 100 50 $tc 0 5)" >> gpurun_out/dropin_sets.log || exit $?
  done
done
echo dropin-done
exit 0
