#!/bin/bash
# no-record sweeps/s under several runtime environment settings (one line each)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for e in "$@"; do
  env HMSC_DIAG_TIMING=1 $e timeout -k 10 100 python -u scripts/norec_rate.py > gpurun_out/envs.log 2>&1 || { echo "FAIL $e"; tail -3 gpurun_out/envs.log; continue; }
  echo "== $e"; grep -E "no record|enqueued" gpurun_out/envs.log | tail -2
done
