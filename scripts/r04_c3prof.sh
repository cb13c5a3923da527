#!/bin/bash
# config 3 (phylogeny + GammaEta) under the kernel trace: per-launch durations of the blocked
# Cholesky steps and the solves
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04_c3}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG -o run -- python $R/bench.py --workload phylo --steps 20 --warmup 200 --no-cpu > $R/gpurun_out/${TAG}_bench.json 2> $R/gpurun_out/$TAG.err || { echo "rocprof failed"; tail -20 $R/gpurun_out/$TAG.err; exit 1; }
python -c "import json;d=json.load(open('$R/gpurun_out/${TAG}_bench.json'));print('config3', d['value'], d.get('kernels_eager_events_us'))"
