#!/bin/bash
# Round-3 session 2: z-kernel part costs (MODE bits, draw parts) and the fixed cost of one run call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s8}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 120 ./scripts/ubench_z > gpurun_out/${TAG}_ubz.log 2>&1 || { echo "ubench_z failed"; tail gpurun_out/${TAG}_ubz.log; exit 1; }
cat gpurun_out/${TAG}_ubz.log
timeout -k 10 120 ./scripts/ubench_parts > gpurun_out/${TAG}_parts.log 2>&1 || { echo "ubench_parts failed"; tail gpurun_out/${TAG}_parts.log; exit 1; }
cat gpurun_out/${TAG}_parts.log
HMSC_DIAG_TIMING=1 timeout -k 10 300 python -u scripts/run_overhead.py > gpurun_out/${TAG}_overhead.log 2>&1 || { echo "overhead failed"; tail -20 gpurun_out/${TAG}_overhead.log; exit 1; }
cat gpurun_out/${TAG}_overhead.log
timeout -k 10 200 python scripts/stamps_sweep.py > gpurun_out/${TAG}_stamps.log 2>&1 || { echo "stamps failed"; tail gpurun_out/${TAG}_stamps.log; exit 1; }
cat gpurun_out/${TAG}_stamps.log
