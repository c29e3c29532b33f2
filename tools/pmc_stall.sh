set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/stall
cd /tmp && export TMPDIR=/tmp
i=0
for g in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_IFETCH" "SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SALU SQ_INSTS_VALU" "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d $R/gpurun_out/stall/p$i -o run -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-dropin --service 0 > $R/gpurun_out/stall/p$i.log 2>&1
  echo "pass $i rc=$?"
done
