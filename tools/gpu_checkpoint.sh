#!/bin/bash
# Round checkpoint on one GPU box: full GPU tests, smoke, the bench line,
# the 16-window ratio gate, rocprofv3 kernel stats of the bench and of C1 /
# C2 / C4 (the PMC HBM traffic passes: tools/gpu_checkpoint_pmc.sh).
#   usage: tools/gpu_checkpoint.sh TAG
set -e
TAG=${1:-ck}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
tail -1 gpurun_out/${TAG}_bench.log
# the 16-window ratio gate of this build (one gate log per checkpoint)
timeout -k 10 300 python3 tools/ratio_gate.py > gpurun_out/${TAG}_gate.log 2>&1
tail -1 gpurun_out/${TAG}_gate.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api --no-per-generator > $R/gpurun_out/${TAG}_prof.log 2>&1
cd $R
cp gpurun_out/${TAG}_prof/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats.csv
cut -d, -f1-4 gpurun_out/${TAG}_kernel_stats.csv | head -14
# secondary configs: C1 (checksums, 1 GiB device-resident), C2 (4096-stream
# batch inflate), C4 (10 000-file GZip batch, host buffers) with kernel stats
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_c1prof -o run -- python3 $R/tools/ck_time.py > $R/gpurun_out/${TAG}_c1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_c2prof -o run -- python3 $R/tools/c2_bench.py 3 > $R/gpurun_out/${TAG}_c2.log 2>&1
cd $R
timeout -k 10 300 python3 tools/c4_batch.py 10000 gpurun_out/${TAG}_c4_batch.json > gpurun_out/${TAG}_c4.log 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${TAG}_c4prof -o run -- python3 $R/tools/c4_batch.py 10000 > $R/gpurun_out/${TAG}_c4prof.log 2>&1
cd $R
for c in c1 c2 c4; do cp gpurun_out/${TAG}_${c}prof/run_kernel_stats.csv gpurun_out/${TAG}_${c}_kernel_stats.csv; done
tail -1 gpurun_out/${TAG}_c1.log; tail -1 gpurun_out/${TAG}_c2.log | cut -c1-300; tail -3 gpurun_out/${TAG}_c4.log | cut -c1-300
