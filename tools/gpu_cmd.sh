set -e
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k deflate > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -1 gpurun_out/t2.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/p7 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/p7.log 2>&1
cd $GRAFT_REPO_ROOT; cut -d, -f1-4 gpurun_out/p7/run_kernel_stats.csv | cut -c1-120 | head -9; grep metric gpurun_out/p7.log | cut -c 1-170
