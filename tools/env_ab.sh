#!/bin/bash
# GPU-box bench A/B of runtime tuning variables on the default bench, two rounds
# interleaved (BENCH_ARGS: extra bench arguments).  Usage: tools/env_ab.sh "SPT_CLAIM=512" ...
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do for v in "NONE=0" "$@"; do
  env "$v" timeout -k 10 200 python bench.py --no-dropin --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/env.tmp 2>&1 || { tail -5 gpurun_out/env.tmp; exit 1; }
  python -c "
import json
for l in open('gpurun_out/env.tmp'):
  if l.startswith('{'): d=json.loads(l); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a gpurun_out/env.log
done; done
