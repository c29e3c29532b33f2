# GPU session: -m gpu suite, VALU issue rates, A/B of $VARIANTS, drop-in batch sets,
# LDS/SALU counters, task-mode bench, PC sampling (last: beta).  A failed step ends it.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest --maxfail=3 -q --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/s3_tests.log 2>&1 || exit $?
tail -1 gpurun_out/s3_tests.log
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/ubench/issue_rates.hip -o /tmp/issue_rates > /dev/null 2>&1 || exit 5
timeout -k 10 60 /tmp/issue_rates > gpurun_out/ubench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --mode task --no-cpu-baseline --no-dropin > gpurun_out/s3_task.log 2>&1 || exit $?
VARIANTS="$VARIANTS" CONFIGS="${CONFIGS:-c2}" bash tools/gpu_ab.sh > gpurun_out/ab.log 2>&1 || exit $?
H=simplepathtracer_amd/lib/spt_dropin_harness
: > gpurun_out/dropin_sets.log
for k in 2 3 4; do
  for t in 0 1; do
    echo "sets=$k task=$t $(SPT_BATCH_SETS=$k timeout -k 10 120 $H /dev/null 1200 800 100 50 4 $t 5)" >> gpurun_out/dropin_sets.log || exit $?
  done
done
bash tools/pmc_lds.sh || exit $?
exit 0
