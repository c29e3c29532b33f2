#!/bin/bash
# GPU session: tools/scaling_probe.py over (streams, SPT_BLOCKS_PER_CU) pairs given as
# "s:b" in $PAIRS (b = 0: the default grid rule).  A failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for p in $PAIRS; do
  s=${p%%:*}; b=${p#*:}
  if [ "$b" = 0 ]; then env_b=""; else env_b="SPT_BLOCKS_PER_CU=$b"; fi
  env $env_b timeout -k 10 200 python tools/scaling_probe.py --streams $s --reps ${REPS:-5} > gpurun_out/sp.log 2>&1 || { tail -5 gpurun_out/sp.log; exit 1; }
  echo "== streams $s blocks/CU $b"; grep "^N=" gpurun_out/sp.log
done
