# GPU session: -m gpu suite, refill/group A/B on config 5, claim sizes on config 5.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest --maxfail=3 -q --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/s10_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s10_tests.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="r8 r24 r32 g1" CONFIGS="c5" ROUNDS=3 bash tools/gpu_ab.sh > gpurun_out/ab10.log 2>&1 || exit $?
: > gpurun_out/claim5.log
for c in 0 192 384 0; do
  echo "claim=$c $(SPT_CLAIM=$c timeout -k 10 200 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline | tail -1 | cut -c1-200)" >> gpurun_out/claim5.log || exit $?
done
exit 0
