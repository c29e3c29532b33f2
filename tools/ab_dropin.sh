#!/bin/bash
# A/B of the drop-in path's launch sharing (SPT_HOST_GRID_DIV) under
# RenderImageParallelMain tiling: config 2, tc = 4 and 8, segment and task mode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
H=simplepathtracer_amd/lib/spt_dropin_harness
for div in ${DIVS:-1 0}; do
  for tc in ${TCS:-4 8}; do
    for task in 0 1; do
      r=$(SPT_HOST_GRID_DIV=$div timeout -k 10 120 $H /dev/null 1200 800 100 50 $tc $task 5) || exit $?
      sec=${r#*seconds=}
      python3 -c "print('div=$div tc=$tc task=$task', round(1200*800*100*5/$sec/1e6, 1), 'Msamples/s')"
    done
  done
done
