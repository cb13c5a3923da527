#!/bin/bash
# bench.py (no CPU baseline) at several sweeps-per-graph-replay settings (HMSC_GRAPH_SWEEPS)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for g in ${@:-4 8 16}; do
  export HMSC_GRAPH_SWEEPS=$g
  timeout -k 10 150 python -u $R/bench.py --steps 320 --warmup 32 --no-cpu --ess-samples 1000 > $R/gpurun_out/gs_$g.json 2> $R/gpurun_out/gs_$g.err || exit 1
  python -c "import json; d=json.load(open('$R/gpurun_out/gs_$g.json')); print('graph_sweeps $g', d['value'], d['kernels_live_us'])"
done
