#!/bin/bash
# Instruction-fetch counters of the sweep's kernels (one rocprofv3 --pmc pass, kernel trace only).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc_icache}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $R/gpurun_out/$TAG/avail.txt 2>&1 || true
grep -i -E "icache|ifetch|SQC_" $R/gpurun_out/$TAG/avail.txt | head -40 > $R/gpurun_out/$TAG/avail_icache.txt || true
HMSC_SIDE_EDGES=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${PMC:-SQ_IFETCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY} \
  --kernel-include-regex "z_wave|eta_fused|gamma2_bl|side_chain|slab_pack" --output-format csv \
  -d $R/gpurun_out/$TAG/p1 -o p -- python $R/scripts/trace_sweeps.py > $R/gpurun_out/$TAG/p1.log 2>&1 || { echo "pass failed"; tail -20 $R/gpurun_out/$TAG/p1.log; exit 1; }
echo pmc done
