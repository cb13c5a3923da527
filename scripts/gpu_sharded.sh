#!/bin/bash
# GPU-box helper: where the species-sharded chain's sweep goes.  Live
# launch-timer timelines (scripts/kt_timeline.py) of the unsharded chain, the one-rank RCCL
# sharded chain at ns = 1000 and at ns = 125 (config 4's 8-way per-rank share), and a rocprofv3
# kernel trace of the sharded chain (scripts/trace_sharded.py) printed per sweep.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-shard}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 200 python -u scripts/kt_timeline.py --record > gpurun_out/${TAG}_kt_unsharded.txt 2>&1 || { cat gpurun_out/${TAG}_kt_unsharded.txt; exit 1; }
timeout -k 10 200 python -u scripts/kt_timeline.py --record --sharded > gpurun_out/${TAG}_kt_sharded.txt 2>&1 || { cat gpurun_out/${TAG}_kt_sharded.txt; exit 1; }
timeout -k 10 200 python -u scripts/kt_timeline.py --record --sharded --ns 125 > gpurun_out/${TAG}_kt_sharded125.txt 2>&1 || { cat gpurun_out/${TAG}_kt_sharded125.txt; exit 1; }
timeout -k 10 200 python -u scripts/kt_timeline.py --record --ns 125 > gpurun_out/${TAG}_kt_unsharded125.txt 2>&1 || { cat gpurun_out/${TAG}_kt_unsharded125.txt; exit 1; }
for f in kt_unsharded kt_sharded kt_sharded125 kt_unsharded125; do echo "== $f"; cat gpurun_out/${TAG}_$f.txt; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_trace -o run -- python $R/scripts/trace_sharded.py > $R/gpurun_out/${TAG}_trace.log 2>&1 || { echo "trace failed"; tail -20 $R/gpurun_out/${TAG}_trace.log; exit 1; }
cd $R
f=$(find gpurun_out/${TAG}_trace -name '*kernel_trace.csv' | head -1)
python scripts/trace_view.py $f gamma2_bl_kernel 3 100 > gpurun_out/${TAG}_trace_view.txt 2>&1
cat gpurun_out/${TAG}_trace_view.txt
