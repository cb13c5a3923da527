#!/bin/bash
# Same-box A/B of environment settings: bench.py (config 4, STEPS steps) alternately under each
# setting given on the command line ("-" = none, else VAR=value[,VAR=value]), ROUNDS rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
ROUNDS=${ROUNDS:-2}
STEPS=${STEPS:-1000}
mkdir -p $R/gpurun_out/ab
for r in $(seq 1 $ROUNDS); do
  i=0
  for setting in "$@"; do
    i=$((i+1))
    envs=()
    [ "$setting" != "-" ] && IFS=, read -ra envs <<< "$setting"
    env "${envs[@]}" timeout -k 10 200 python -u $R/bench.py --steps $STEPS --warmup ${WARMUP:-100} --no-cpu --no-sharded-leg \
      > $R/gpurun_out/ab/env$i.$r.json 2> $R/gpurun_out/ab/env$i.$r.err || { echo "bench failed: $setting"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$R/gpurun_out/ab/env$i.$r.json').read().strip().splitlines()[-1])
print('$setting', $r, d['value'], d['kernels_live_us'])"
  done
done
