#!/bin/bash
# GPU-box helper (round 6): the GPU suite, then the driver-shaped 20-step line A/B'd over
# run-shape settings (ROUNDS rounds), then one 20-step line with the library's host timer.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest.log | head -30
tail -2 gpurun_out/${TAG}_pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit 1;; esac
ROUNDS=${ROUNDS:-3} STEPS=20 WARMUP=5 bash scripts/ab_env.sh "$@" || exit 1
HMSC_DIAG_TIMING=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-sharded-leg > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_b20.json').read().strip().splitlines()[-1]); print('b20', d['value'], d['ms_per_step'])"
grep "run 20 sweeps" gpurun_out/${TAG}_b20.err | head -2
