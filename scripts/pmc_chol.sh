#!/bin/bash
# Kernel trace + PMC passes (one counter group per rocprofv3 run) over the standalone blocked
# Cholesky at the config-5 size: MFMA instruction counts / busy cycles of the factorization.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc_chol}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG/kt -o p -- \
  python3 $R/scripts/chol_bench.py 5000 3 > $R/gpurun_out/$TAG/kt.log 2>&1 || { echo "trace failed"; tail -5 $R/gpurun_out/$TAG/kt.log; exit 1; }
i=0
for grp in "SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv \
    -d $R/gpurun_out/$TAG/p$i -o p -- python3 $R/scripts/chol_bench.py 5000 2 > $R/gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/$TAG/p$i.log; exit 1; }
done
echo pmc done
