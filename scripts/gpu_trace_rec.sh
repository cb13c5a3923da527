#!/bin/bash
# GPU-box helper: kernel + memory-copy trace of the recording diagnostic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-rectrace}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $R/gpurun_out/${TAG} -o run -- python $R/scripts/record_overhead.py 1 > $R/gpurun_out/${TAG}.log 2>&1 || { echo "rocprof failed"; tail -20 $R/gpurun_out/${TAG}.log; exit 1; }
cat $R/gpurun_out/${TAG}.log
