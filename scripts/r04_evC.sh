#!/bin/bash
# round 4 evidence C: kernel trace + stats of a 300-step bench run with the side chain behind
# graph edges (HMSC_SIDE_EDGES=1): under the kernel trace the device-side joins see the side
# queue's dispatches late, so the traced durations of the edge-free sweep are not its own
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04_s3}
cd /tmp && export TMPDIR=/tmp
HMSC_SIDE_EDGES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_profedges -o run -- python $R/bench.py --steps 300 --warmup 30 --no-cpu > $R/gpurun_out/${TAG}_profedges_bench.json 2> $R/gpurun_out/${TAG}_profedges.err || { echo "rocprof failed"; tail -20 $R/gpurun_out/${TAG}_profedges.err; exit 1; }
cd $R
HMSC_SIDE_EDGES=1 timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_edges_bench.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/${TAG}_edges_bench.json'));print('edges 1000', d['value'], d['kernels_live_us'])"
python -c "import json;d=json.load(open('gpurun_out/${TAG}_profedges_bench.json'));print('edges traced', d['value'], d['kernels_live_us'])"
echo done
