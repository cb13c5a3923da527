#!/bin/bash
# A/B on one box: bench.py with and without the per-sweep hipGraph, twice each, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
for rep in 1 2; do
  for ng in 0 1; do
    HMSC_NO_GRAPH=$ng timeout -k 10 300 python bench.py --steps ${STEPS:-300} --warmup 30 --no-cpu > gpurun_out/ab_${ng}_${rep}.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_${ng}_${rep}.json')); print('no_graph=$ng', d['value'], d['ms_per_step'], d['kernels_us'])"
  done
done
