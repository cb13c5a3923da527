#!/bin/bash
# Same-box A/B of library builds: bench.py (config 4, 1000 steps) alternately with each .so
# given on the command line (HMSC_AMD_LIB), ROUNDS rounds; prints value and live z / eta / BL.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
ROUNDS=${ROUNDS:-2}
STEPS=${STEPS:-1000}
mkdir -p $R/gpurun_out/ab
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    HMSC_AMD_LIB=$R/$lib timeout -k 10 200 python -u $R/bench.py --steps $STEPS --warmup 100 --no-cpu --no-sharded-leg \
      > $R/gpurun_out/ab/$tag.$r.json 2> $R/gpurun_out/ab/$tag.$r.err || { echo "bench failed: $lib"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$R/gpurun_out/ab/$tag.$r.json').read().strip().splitlines()[-1])
print('$tag', $r, d['value'], d['kernels_live_us'])"
  done
done
