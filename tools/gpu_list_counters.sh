#!/bin/bash
# the TCC / EA counters rocprofv3 offers on this box
mkdir -p gpurun_out/calib
cd /tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/calib/list.txt 2>&1 || true
cd $GRAFT_REPO_ROOT
grep -o "TCC_EA0_RD[A-Z0-9_]*\|TCC_EA0_WR[A-Z0-9_]*\|TCC_BUBBLE[A-Z0-9_]*\|TCC_REQ[A-Z0-9_]*" gpurun_out/calib/list.txt | sort -u | head -40
