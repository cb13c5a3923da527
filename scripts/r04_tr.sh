#!/bin/bash
# kernel trace of the current library (bench, 300 steps): per-sweep timeline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-tr}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG -o run -- python $R/bench.py --steps 300 --warmup 30 --no-cpu > $R/gpurun_out/${TAG}_bench.json 2> $R/gpurun_out/$TAG.err || { echo "rocprof failed"; tail -20 $R/gpurun_out/$TAG.err; exit 1; }
cd $R && python scripts/trace_timeline.py gpurun_out/$TAG/run_kernel_trace.csv | head -14
