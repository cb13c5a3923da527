#!/bin/bash
# GPU-box helper: kernel + HIP API trace of the no-record rate script (env passed through).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-nr}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG} -o run -- python $R/scripts/norec_rate.py > $R/gpurun_out/${TAG}.log 2>&1 || { echo "rocprof failed"; tail -20 $R/gpurun_out/${TAG}.log; exit 1; }
grep "no record" $R/gpurun_out/${TAG}.log
