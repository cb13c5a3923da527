#!/bin/bash
# bench.py (no CPU baseline) at several z-grid site-chunk counts (HMSC_Z_CHUNKS)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for c in ${@:-0 48 64 96 157}; do
  if [ "$c" = "0" ]; then unset HMSC_Z_CHUNKS; else export HMSC_Z_CHUNKS=$c; fi
  timeout -k 10 150 python -u $R/bench.py --steps 300 --warmup 30 --no-cpu --ess-samples 1000 > $R/gpurun_out/zc_$c.json 2> $R/gpurun_out/zc_$c.err || exit 1
  python -c "import json; d=json.load(open('$R/gpurun_out/zc_$c.json')); print('chunks $c', d['value'], d['kernels_live_us'])"
done
