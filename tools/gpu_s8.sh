# GPU session: leaf-pass threshold / budget sweep around the 6-step lane walk (config 5,
# 20k spheres), then the kernel trace of the drop-in at tc = 4.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
VARIANTS="t48 t56 t32 s6b10 s6b6 s5b9" CONFIGS="c5 s20k" ROUNDS=3 bash tools/gpu_ab.sh > gpurun_out/ab8.log 2>&1 || exit $?
bash tools/trace_dropin.sh || exit $?
exit 0
