#!/bin/bash
# GPU-box helper: kernel trace of a short bench run (extra env passed through), e.g.
#   HMSC_NO_GRAPH=1 bash scripts/gpu_trace_bench.sh tag
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-tb}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG} -o run -- python $R/bench.py --steps ${STEPS:-200} --warmup 30 --no-cpu > $R/gpurun_out/${TAG}.json 2> $R/gpurun_out/${TAG}.err || { echo "rocprof failed"; tail -20 $R/gpurun_out/${TAG}.err; exit 1; }
cat $R/gpurun_out/${TAG}.json
