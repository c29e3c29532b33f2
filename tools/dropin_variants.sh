H=./simplepathtracer_amd/lib/spt_dropin_harness
for tc in 4 32; do
  for v in "SPT_SERVICE=0" "SPT_SERVICE=1" "SPT_SERVICE=1 SPT_BATCH=0" "SPT_SERVICE=1 SPT_BATCH_SETS=4" "SPT_SERVICE=1 SPT_BATCH_SETS=8" "SPT_SERVICE=0 SPT_BATCH_SETS=4"; do
    echo "tc=$tc $v: $(env $v timeout -k 10 120 $H /dev/null 1200 800 100 50 $tc 0 5 | cut -c1-60)"
  done
done
