#!/bin/bash
# GPU-box helper: kernel + memory-copy trace of a recorded run (record_overhead.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-rt}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/${TAG} -o run -- python $R/scripts/record_overhead.py 2 > $R/gpurun_out/${TAG}.log 2>&1 || { echo "rocprof failed"; tail -20 $R/gpurun_out/${TAG}.log; exit 1; }
grep record $R/gpurun_out/${TAG}.log
