# GPU session: HEAD profiles of configs 2 and 5, wavefront engine benches, 4-rank
# gloo rehearsal of bench.py --gpus 4 (one GPU).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
bash tools/profile.sh r03b_c2 c2 || exit $?
bash tools/profile.sh r03b_c5 c5 --config c5 --steps 4 --warmup 1 --no-cpu-baseline || exit $?
timeout -k 10 200 python bench.py --engine wavefront --steps 5 --no-cpu-baseline --no-dropin > gpurun_out/wf_c2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --engine wavefront --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/wf_c5.log 2>&1 || exit $?
timeout -k 10 300 env SPT_DIST_BACKEND=gloo python bench.py --gpus 4 --steps 3 --warmup 1 --no-cpu-baseline --no-dropin --dump gpurun_out/g4.bin > gpurun_out/g4.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dropin --dump gpurun_out/g1.bin > gpurun_out/g1.log 2>&1 || exit $?
cmp gpurun_out/g1.bin gpurun_out/g4.bin && echo "g4 == g1" > gpurun_out/g4cmp.log
rm -f gpurun_out/g1.bin gpurun_out/g4.bin
exit 0
