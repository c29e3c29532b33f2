# LDS pressure of the lane walk (config 5) and the wave walk (config 2): one --pmc pass each.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/lds"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS \
  --output-format csv -d "$OUT/c5" -o run -- python3 "$R/bench.py" --config c5 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c5.log" 2>&1 || exit $?
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INST_CYCLES_SALU \
  --output-format csv -d "$OUT/c2" -o run -- python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline --no-dropin > "$OUT/c2.log" 2>&1
exit 0
