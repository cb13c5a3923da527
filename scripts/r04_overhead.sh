#!/bin/bash
# run-overhead probe of the 20-sweep recorded run (the driver's bench line) under a few settings
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r04_overhead.log
: > $out
for cfg in "" "HMSC_GRAPH_SWEEPS=8" "HMSC_UNPACK_THREADS=8"; do
  echo "== $cfg" >> $out
  env $cfg HMSC_DIAG_TIMING=1 timeout -k 10 120 python -u scripts/run_overhead.py 20 >> $out 2>&1 || exit $?
done
