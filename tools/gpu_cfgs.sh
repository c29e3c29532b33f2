# GPU session: the full-size configs through bench.py (c3, c5, task-mode c2) and the
# driver's default command (c2 with the CPU baseline and the drop-in legs)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cfg
mkdir -p $O
timeout -k 10 200 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3.log 2>&1 && \
timeout -k 10 200 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1 && \
timeout -k 10 200 python bench.py --mode task --no-cpu-baseline --no-dropin > $O/c2task.log 2>&1 && \
timeout -k 10 200 python bench.py --config c1 --steps 50 --no-cpu-baseline > $O/c1.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/c2.log 2>&1
