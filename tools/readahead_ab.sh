#!/bin/bash
# Drop-in read-ahead A/B: the C++ harness at tc = 4 (segment, task), 20 frames, per setting.
H=./simplepathtracer_amd/lib/spt_dropin_harness
for r in 1 2; do
for v in "SPT_READAHEAD=0" "SPT_READAHEAD_PARTS=4" "SPT_READAHEAD_PARTS=8"; do
  for task in 0 1; do
    s=$(env $v timeout -k 10 60 $H /dev/null 1200 800 100 50 4 $task 20 | grep -o "seconds=[0-9.]*" | cut -d= -f2)
    echo "r$r $v task=$task: $(python3 -c "print(f'{$s/20*1e3:.3f} ms/frame, {1200*800*100*20/$s/1e6:.0f} Msamples/s')")"
  done
done
done
export TMPDIR=/tmp
timeout -k 10 100 rocprofv3 --kernel-trace -d gpurun_out/rat -o rat -- $H /dev/null 1200 800 100 50 4 0 3 > gpurun_out/rat.log 2>&1
