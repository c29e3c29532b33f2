#!/bin/bash
# Round-4 A/B experiments (GPU box), one named experiment per call; every run under its own
# time limit, two interleaved rounds where timing noise matters.  The results are quoted in
# DESIGN.md (section in brackets).
#   claims        launch-path claim size, config-2 bench line (SPT_CLAIM)            [§7]
#   c5claims      config-5 claim size, bench ms per frame                            [§7]
#   c5write       config-5 render WRITE_SIZE per launch against the claim size        [§9]
#   svc           service settings on the bench line and the 1/8 share probe           [§4.7]
#   svctimeline   service variants: per-frame completion slope and intercept
#                 (libraries from `make variants`; edit VARIANTS below)               [§5]
#   dropin        drop-in harness: service, batching and read-ahead settings at tc 4/32 [§5, §9]
#   readahead     drop-in harness at tc = 4: read-ahead off / parts                    [§5]
# Usage: tools/experiments.sh <name>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
H=./simplepathtracer_amd/lib/spt_dropin_harness
val() { grep -o "$1" | tr '\n' ' '; }
case ${1:?experiment} in
  claims)
    for r in 1 2; do for c in "" 640 896 1344; do
      echo "r$r claim=${c:-auto}: $(SPT_CLAIM=$c timeout -k 10 120 python bench.py --no-cpu-baseline --no-dropin --service 0 2>&1 | val '"value": [0-9.]*')"
    done; done ;;
  c5claims)
    for r in 1 2; do for c in "" 512 1024; do
      echo "r$r claim=${c:-auto}: $(SPT_CLAIM=$c timeout -k 10 200 python bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline --no-dropin 2>&1 | val '"ms_per_step": [0-9.]*')"
    done; done ;;
  c5write)
    cd /tmp && export TMPDIR=/tmp
    for c in "" 128 512 1024; do
      d="$R/gpurun_out/c5w_${c:-def}"
      SPT_CLAIM=$c timeout -k 10 -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$d" -o run -- \
        python3 "$R/bench.py" --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin > "$d.log" 2>&1 || exit $?
      python3 - "$d" "${c:-def}" <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
v = [float(r["Counter_Value"]) for r in rows if "render_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE"]
print(f"claim {sys.argv[2]}: WRITE_SIZE per launch (KiB) {[round(x) for x in v]}")
PY
    done ;;
  svc)
    B="python bench.py --no-cpu-baseline --no-dropin"
    for r in 1 2; do
      echo "r$r svc0: $(timeout -k 10 120 $B --service 0 2>&1 | val '"value": [0-9.]*')"
      echo "r$r svc1: $(timeout -k 10 120 $B --service 1 2>&1 | val '"value": [0-9.]*')"
      echo "r$r svc1 wt0: $(SPT_LIB=libspt_hip_wt0.so timeout -k 10 120 $B --service 1 2>&1 | val '"value": [0-9.]*')"
      for c in 896 256; do echo "r$r svc1 claim$c: $(SPT_SVC_CLAIM=$c timeout -k 10 120 $B --service 1 2>&1 | val '"value": [0-9.]*')"; done
    done
    P="python tools/scaling_probe.py --streams 2 --reps 3 --ns 8"
    for s in 0 1; do echo "n8 svc$s: $(timeout -k 10 120 $P --service $s 2>&1 | val 'wall per frame *[0-9.]* ms')"; done
    for st in 8 20; do echo "n8 svc1 strip$st: $(timeout -k 10 120 $P --service 1 --strip $st 2>&1 | val 'wall per frame *[0-9.]* ms')"; done ;;
  svctimeline)
    VARIANTS=${VARIANTS:-"libspt_hip.so"}
    for v in $VARIANTS; do for n in 8 1; do
      echo "$v n=$n: $(SPT_LIB=$v timeout -k 10 120 python tools/svc_timeline.py --n $n --reps 2 2>&1 | val 'wall [0-9.]* ms\|slope [0-9.]* ms/frame, intercept [0-9.]* ms')"
    done; done
    for n in 8 1; do
      echo "launches n=$n: $(timeout -k 10 120 python tools/svc_timeline.py --n $n --reps 2 --service 0 2>&1 | val 'wall [0-9.]* ms\|slope [0-9.]* ms/frame, intercept [0-9.]* ms')"
    done ;;
  dropin)
    for tc in 4 32; do for v in "SPT_READAHEAD=0" "SPT_READAHEAD=0 SPT_SERVICE=1" "SPT_READAHEAD=0 SPT_SERVICE=1 SPT_BATCH=0" \
                                "SPT_READAHEAD=0 SPT_SERVICE=1 SPT_BATCH_SETS=4" "SPT_READAHEAD=1"; do
      echo "tc=$tc $v: $(env $v timeout -k 10 120 $H /dev/null 1200 800 100 50 $tc 0 5 | cut -c1-60)"
    done; done ;;
  readahead)
    for r in 1 2; do for v in "SPT_READAHEAD=0" "SPT_READAHEAD_PARTS=4" "SPT_READAHEAD_PRIO=-1" "SPT_READAHEAD_PRIO=1"; do for task in 0 1; do
      s=$(env $v timeout -k 10 60 $H /dev/null 1200 800 100 50 4 $task 20 | grep -o "seconds=[0-9.]*" | cut -d= -f2)
      echo "r$r $v task=$task: $(python3 -c "print(f'{$s/20*1e3:.3f} ms/frame, {1200*800*100*20/$s/1e6:.0f} Msamples/s')")"
    done; done; done ;;
  *) echo "unknown experiment $1"; exit 2 ;;
esac
