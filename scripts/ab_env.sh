#!/bin/bash
# A/B on one box: bench.py under two environment settings, interleaved, twice each.
#   bash scripts/ab_env.sh "HMSC_GRAPH_EXECS=1" "HMSC_GRAPH_EXECS=2"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
for rep in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python bench.py --steps ${STEPS:-1000} --warmup 30 --no-cpu > gpurun_out/abe_${i}_${rep}.json 2>gpurun_out/abe.err || { tail -5 gpurun_out/abe.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abe_${i}_${rep}.json')); print('$e', d['value'], d['ms_per_step'])"
  done
done
