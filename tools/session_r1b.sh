#!/bin/bash
# GPU-box session: GPU tests + smoke + bench (tools/gpu_session.sh), the SPT_DIAG
# counters of config 2, an A/B of traversal shapes, then the rocprofv3 profile.
# Usage: tools/session_r1b.sh <profile tag>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
bash tools/gpu_session.sh || exit $?
make -s -C simplepathtracer_amd/csrc diag > gpurun_out/diag_build.log 2>&1 || { tail gpurun_out/diag_build.log; exit 3; }
echo "== diag c2"
SPT_LIB=libspt_hip_diag.so timeout -k 10 180 python tools/diag.py c2 > gpurun_out/diag_c2.log 2>&1
rc=$?; cat gpurun_out/diag_c2.log; [ $rc -eq 0 ] || exit $rc
echo "== ab shapes"
timeout -k 10 300 python tools/ab.py libspt_hip.so libspt_hip.so:8:4 libspt_hip.so:8:2 libspt_hip.so:8 --rounds 3 \
  > gpurun_out/ab_shapes.log 2>&1
rc=$?; cat gpurun_out/ab_shapes.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile.sh "${1:-prof}"
