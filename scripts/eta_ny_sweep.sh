#!/bin/bash
# Eta's live duration against ny (tiles of 16 sites: 512 = 2 per CU, 625, 768 = 3 per CU).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/etany
for ny in 8192 10000 12288; do
  timeout -k 10 200 python -u $R/bench.py --ny $ny --steps 400 --warmup 100 --no-cpu --no-sharded-leg \
    > $R/gpurun_out/etany/ny$ny.json 2> $R/gpurun_out/etany/ny$ny.err || { echo "bench failed: $ny"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$R/gpurun_out/etany/ny$ny.json').read().strip().splitlines()[-1])
print($ny, d['value'], d['kernels_live_us'])"
done
