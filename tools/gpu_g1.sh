# GPU session: the -m gpu suite, then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest --maxfail=5 -v --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/g1_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-dropin > gpurun_out/g1_bench.log 2>&1
