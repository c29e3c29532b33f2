# PC sampling of the config-2 render kernel (rocprofv3 beta, host trap, time unit):
# which instructions the waves sit on.  One short bench run, killed after 120 s.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pcs"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${PCS_METHOD:-host_trap} \
  --pc-sampling-unit ${PCS_UNIT:-time} --pc-sampling-interval ${PCS_INTERVAL:-1} --output-format csv -d "$OUT" -o run \
  -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/run.log" 2>&1
rc=$?
echo "rc=$rc"; tail -5 "$OUT/run.log"; find "$OUT" -type f | head -20
exit $rc
