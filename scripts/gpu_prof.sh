#!/bin/bash
# GPU-box helper: rocprofv3 kernel trace + stats of a short bench run (no CPU baseline).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG} -o run -- python $R/bench.py --steps ${STEPS:-200} --warmup 30 --no-cpu > $R/gpurun_out/${TAG}_bench.json 2> $R/gpurun_out/${TAG}.err || { echo "rocprof failed"; tail -20 $R/gpurun_out/${TAG}.err; exit 1; }
cat $R/gpurun_out/${TAG}_bench.json
