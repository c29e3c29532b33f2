#!/bin/bash
# GPU-box check of the current tree: GPU tests, smoke, bench lines of every config
# (config 2 in both modes).  Usage: tools/session_check.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 1 "gpurun_out/$name.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "stop $name rc=$rc"; exit $rc; }; }
run gpu_tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench_c2 300 python bench.py
run bench_c2_task 200 python bench.py --mode task --no-dropin --no-cpu-baseline
run bench_c1 200 python bench.py --config c1 --steps 20 --warmup 3
run bench_c3 300 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline
run bench_c5 300 python bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline
