#!/bin/bash
# GPU-box session runner: named steps, each under its own time limit, logs under
# gpurun_out/<tag>_<step>.log.  A timeout, abort, segfault or kill ends the session (no
# further GPU step runs after a possible fault); a step that merely fails (tests red,
# nonzero exit) is reported and the next step runs.
# Usage: tools/session.sh <tag> <step> [<step> ...]
#   steps: svc          pytest tests/test_gpu_service.py
#          gpu          pytest -m gpu (the whole GPU suite)
#          mr           bench.py --gpus 2 rehearsals (gloo ranks on one GPU, launches and service)
#          smoke        __graft_entry__.smoke()
#          bench        python bench.py (default arguments: config 2, service on)
#          bench0       python bench.py --service 0 (one launch per frame)
#          benchq       bench.py without the CPU baseline and drop-in legs (quick)
#          bench0q      the same with --service 0
#          c5 / c3      bench.py --config c5 / c3 (quick legs)
#          scaling      tools/scaling_probe.py --streams 2 (service on and off)
#          dropin       the C++ drop-in harness at tc = 4 and tc = 32 (bench.py's legs)
#          dropin1      the same with SPT_SERVICE=1 (the shim's calls through the render service)
#          profile      tools/profile.sh <tag>_c2 c2 (kernel trace + PMC passes + SPT_DIAG)
#          profile5     tools/profile.sh <tag>_c5 c5 --config c5 --steps 2 --warmup 1 ...
#          profile3     the same for config 3 (3840x2160, 1024 spp)
#          tdrop        tools/trace_dropin.sh (kernel trace of the C++ drop-in at tc = 4)
#          attrib       tools/attrib.sh (per-phase VALU from the SPT_DUP builds)
#          benchenv:V=X,W=Y  benchq with those environment variables (logs benchenv1, 2, ...)
#          ab:<args>    tools/ab.py <args> (one quoted step; logs ab1, ab2, ...)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
mkdir -p gpurun_out
TAG=${1:?tag}
shift
run() {  # name seconds cmd...
  local name=$1 t=$2; shift 2
  local log="$R/gpurun_out/${TAG}_${name}.log"
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 6 "$log"
  case $rc in 124|134|137|139) echo "stopping after $name (rc=$rc)"; exit $rc ;; esac
  return 0
}
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
for step in "$@"; do
  case $step in
    svc) run svc 300 $PYT -v tests/test_gpu_service.py ;;
    gpu) run gpu 600 $PYT -m gpu tests ;;
    svcdbg) SPT_SVC_DEBUG=1 run svcdbg 300 python -u -m pytest -x -v -s --timeout 90 --timeout-method thread tests/test_gpu_service.py ;;
    rw0) SPT_SVC_DEBUG=1 SPT_TEST_BLOCK_US=0 run rw0 120 python -u -m pytest -x -v -s --timeout 60 --timeout-method thread tests/test_gpu_service.py -k ring_wrap ;;
    rw) SPT_SVC_DEBUG=1 run rw 120 python -u -m pytest -x -v -s --timeout 60 --timeout-method thread tests/test_gpu_service.py -k ring_wrap ;;
    diag) SPT_LIB=libspt_hip_diag.so run diag 200 python tools/diag.py c2 --json "gpurun_out/${TAG}_diag_c2.json" ;;
    diag5) SPT_LIB=libspt_hip_diag.so run diag5 300 python tools/diag.py c5 --json "gpurun_out/${TAG}_diag_c5.json" ;;
    ra) run ra 300 $PYT -v tests/test_gpu_readahead.py ;;
    pl) run pl 300 $PYT -v -m gpu tests/test_gpu_parity.py -k primary_lists ;;
    benchq_nol) SPT_PRIM_LISTS=0 run benchq_nol 120 python bench.py --no-cpu-baseline --no-dropin ;;
    diag5_nol) SPT_PRIM_LISTS=0 SPT_LIB=libspt_hip_diag.so run diag5_nol 300 python tools/diag.py c5 --json "gpurun_out/${TAG}_diag_nol_c5.json" ;;
    trace) (cd /tmp && TMPDIR=/tmp run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_trace" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-dropin) ;;
    diag_nol) SPT_PRIM_LISTS=0 SPT_LIB=libspt_hip_diag.so run diag_nol 200 python tools/diag.py c2 --json "gpurun_out/${TAG}_diag_nol_c2.json" ;;
    mr) run mr 300 $PYT -v -m gpu tests/test_gpu_parity.py -k two_ranks ;;
    smoke) run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python bench.py ;;
    bench1q) run bench1q 120 python bench.py --no-cpu-baseline --no-dropin --service 1 ;;
    bench0) run bench0 400 python bench.py --service 0 ;;
    benchq) run benchq 120 python bench.py --no-cpu-baseline --no-dropin ;;
    bench0q) run bench0q 120 python bench.py --no-cpu-baseline --no-dropin --service 0 ;;
    c5_nol) SPT_PRIM_LISTS=0 run c5_nol 300 python bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline --no-dropin ;;
    c5q) run c5q 300 python bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline --no-dropin ;;
    tl1) run tl1 300 python tools/svc_timeline.py --n 1 --frames 20 --service 1 ;;
    tl0) run tl0 300 python tools/svc_timeline.py --n 1 --frames 20 --service 0 ;;
    bench1q_896) SPT_SVC_CLAIM=896 run bench1q_896 120 python bench.py --no-cpu-baseline --no-dropin --service 1 ;;
    c5) run c5 300 python bench.py --config c5 --steps 4 --warmup 1 --no-cpu-baseline ;;
    c3) run c3 300 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline ;;
    scaling) run scaling 300 python tools/scaling_probe.py --streams 2 --reps 5 --service 1 --record "gpurun_out/${TAG}_scaling.txt"
             run scaling0 300 python tools/scaling_probe.py --streams 2 --reps 5 --service 0 --record "gpurun_out/${TAG}_scaling0.txt" ;;
    dropin) run dropin 300 python -c "import bench; print(bench.dropin_bench(1200, 800, 100, 50, 20, (4, 32)))" ;;
    dropin4) NDI=$((${NDI:-0} + 1)); run dropin4_$NDI 300 python -c "import bench; print(bench.dropin_bench(1200, 800, 100, 50, 20, (4,)))" ;;
    dropinenv:*) NDE=$((${NDE:-0} + 1)); (for kv in $(echo "${step#dropinenv:}" | tr ',' ' '); do export "$kv"; done
                run dropinenv$NDE 300 python -c "import bench; print(bench.dropin_bench(1200, 800, 100, 50, 20, (4,)))") ;;
    dropin1) run dropin1 300 python -c "import bench; print(bench.dropin_bench(1200, 800, 100, 50, 20, (4, 32), {'SPT_SERVICE': '1'}))" ;;
    profile) run profile 900 bash tools/profile.sh "${TAG}_c2" c2 ;;
    profile5) run profile5 900 bash tools/profile.sh "${TAG}_c5" c5 --config c5 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin ;;
    attrib) run attrib 600 bash tools/attrib.sh "${TAG}_attrib" ;;
    benchenv:*) NBE=$((${NBE:-0} + 1)); (for kv in $(echo "${step#benchenv:}" | tr ',' ' '); do export "$kv"; done
                run benchenv$NBE 120 python bench.py --no-cpu-baseline --no-dropin) ;;
    bench1env:*) NB1=$((${NB1:-0} + 1)); (for kv in $(echo "${step#bench1env:}" | tr ',' ' '); do export "$kv"; done
                run bench1env$NB1 120 python bench.py --no-cpu-baseline --no-dropin --service 1) ;;
    tlenv:*) NTL=$((${NTL:-0} + 1)); (for kv in $(echo "${step#tlenv:}" | tr ',' ' '); do export "$kv"; done
                run tlenv$NTL 300 python tools/svc_timeline.py --n 1 --frames 20 --service 1 --reps 2) ;;
    streams3) run streams3 120 python bench.py --no-cpu-baseline --no-dropin --streams 3 ;;
    profile3) run profile3 1100 bash tools/profile.sh "${TAG}_c3" c3 --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin ;;
    tdrop) run tdrop 200 bash tools/trace_dropin.sh ;;
    tdrop20) TDROP_FRAMES=20 run tdrop20 200 bash tools/trace_dropin.sh ;;
    ab:*) NAB=$((${NAB:-0} + 1)); run ab$NAB 600 python tools/ab.py ${step#ab:} ;;
    probe:*) NPR=$((${NPR:-0} + 1)); spec=${step#probe:}; envs=${spec%%|*}; pargs=${spec#*|}
             run probe$NPR 400 env $(echo "$envs" | tr ',' ' ') python tools/scaling_probe.py --streams 2 --reps 3 $pargs \
                 --record "gpurun_out/${TAG}_probe$NPR.txt" ;;
    pyt:*) NPY=$((${NPY:-0} + 1)); run pyt$NPY 400 $PYT -v -s ${step#pyt:} ;;
    benchc:*) NBC=$((${NBC:-0} + 1)); run benchc$NBC 300 python bench.py --no-cpu-baseline --no-dropin --config ${step#benchc:} ;;
    coldtrace) SPT_HOST_TRACE=1 SPT_HARNESS_COLD=2 run coldtrace 120 simplepathtracer_amd/lib/spt_dropin_harness /dev/null 1200 800 100 50 4 0 0 ;;
    dropincold) run dropincold 300 python -c "import bench; print(bench.dropin_bench(1200, 800, 100, 50, 20, (4,)))" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
