#!/bin/bash
# GPU session: parity subset, pow5 fast-path A/B, bench config 2 with 2 / 3 frames in flight
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "numerics or per_sample or config2_every or task_mode" > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py libspt_hip.so libspt_hip_slowpow.so --rounds 6 --config c2 || exit $?
for r in 1 2; do for s in 2 3; do
  timeout -k 10 200 python bench.py --streams $s --no-dropin --no-cpu-baseline | python3 -c "import json,sys; d=json.loads([x for x in sys.stdin if x.startswith('{')][-1]); print('streams $s', d['value'], d['ms_per_step'])" || exit $?
done; done
# drop-in kernel trace with batched folds into the device frame + DMA copy-back
mkdir -p gpurun_out/tdrop0 && cd /tmp && SPT_FOLD_HOST=0 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/tdrop0" -o run -- "$GRAFT_REPO_ROOT/simplepathtracer_amd/lib/spt_dropin_harness" /dev/null 1200 800 100 50 4 0 3 > "$GRAFT_REPO_ROOT/gpurun_out/tdrop0/run.log" 2>&1 || exit $?
