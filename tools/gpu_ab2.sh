#!/bin/bash
# GPU session: sampler-subset parity tests, then A/B of libspt_hip.so vs libspt_hip_old.so on
# configs 2 and 5 (single stream) and the config-2 bench (two frames in flight)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTS:-per_sample or config2_every or task_mode or batched or lane_walk}" > gpurun_out/t.log 2>&1; rc=$?; tail -1 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py libspt_hip.so libspt_hip_old.so --rounds 5 --config c2 || exit $?
[ -n "$NO_C5" ] || timeout -k 10 400 python tools/ab.py libspt_hip.so libspt_hip_old.so --rounds 3 --config c5 || exit $?
VARIANTS=old ROUNDS=3 bash tools/bench_ab.sh
