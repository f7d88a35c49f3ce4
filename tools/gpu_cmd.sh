set -e
export TMPDIR=/tmp
ZT_INF_DEBUG=1 timeout -k 10 300 python tools/inf_debug.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/p5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/p5.log 2>&1
cd $GRAFT_REPO_ROOT; cut -d, -f1-4 gpurun_out/p5/run_kernel_stats.csv | cut -c1-120 | head -8; grep metric gpurun_out/p5.log | cut -c1-200
