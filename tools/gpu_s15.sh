#!/bin/bash
# GPU session: the drop-in path's GPU tests (batched calls, the C++ shim), then an
# interleaved drop-in A/B of $VARIANTS (tools/ab_dropin_libs.sh).  A failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "batch or dropin or shim or concurrent" > gpurun_out/s15_tests.log 2>&1 || { tail -30 gpurun_out/s15_tests.log; exit 1; }
tail -1 gpurun_out/s15_tests.log
VARIANTS="$VARIANTS" ROUNDS=${ROUNDS:-4} TCS="${TCS:-4}" TASK=${TASK:-1} bash tools/ab_dropin_libs.sh > gpurun_out/dab.log 2>&1; rc=$?
python3 - <<'PY'
import collections, re
r = collections.defaultdict(list)
for l in open("gpurun_out/dab.log"):
    m = re.match(r"round \d+ (\S+) (tc=\d+ task=\d) ([\d.]+)", l)
    if m: r[(m.group(1), m.group(2))].append(float(m.group(3)))
for k, v in sorted(r.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    v.sort(); print(k[1], f"{k[0]:40s}", "median", v[len(v)//2], "all", v)
PY
exit $rc
