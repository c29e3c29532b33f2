# GPU session: interleaved A/B of libspt_hip.so against $VARIANTS on $CONFIGS
# (tools/ab.py), optionally the VALU issue-rate microbenchmark first (UBENCH=1)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
if [ -n "$UBENCH" ]; then timeout -k 10 60 tools/ubench/issue_rates > gpurun_out/ubench.log 2>&1 || exit $?; cat gpurun_out/ubench.log; fi
for c in ${CONFIGS:-c2}; do
  libs="libspt_hip.so"; for v in $VARIANTS; do libs="$libs libspt_hip_$v.so"; done
  echo "== ab $c"
  timeout -k 10 400 python tools/ab.py $libs --rounds ${ROUNDS:-4} --config $c || exit $?
done
