#!/bin/bash
# GPU-box bench A/B of libspt_hip variants (SPT_LIB) on the default bench, two rounds
# interleaved.  Build the variants first (make -C simplepathtracer_amd/csrc variants).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do for v in libspt_hip.so libspt_hip_blk128.so libspt_hip_blk64.so libspt_hip_blk512.so; do
  SPT_LIB=$v timeout -k 10 120 python bench.py --no-dropin --no-cpu-baseline > gpurun_out/blk.tmp 2>&1 || { tail -5 gpurun_out/blk.tmp; exit 1; }
  python -c "
import json
for l in open('gpurun_out/blk.tmp'):
  if l.startswith('{'): d=json.loads(l); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a gpurun_out/blk.log
done; done
