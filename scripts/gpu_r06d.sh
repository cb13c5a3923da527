#!/bin/bash
# GPU-box helper (round 6): the GPU suite under an environment setting, then same-box A/B of
# the 20-step and 1000-step lines with and without it.  usage: gpu_r06d.sh TAG VAR=value
# (PYTEST_ENV: the suite's setting instead, e.g. HMSC_NONE=1 for the defaults)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; SET=$2
mkdir -p $R/gpurun_out
cd $R
env ${PYTEST_ENV:-$SET} timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest.log | head -30
tail -2 gpurun_out/${TAG}_pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit 1;; esac
ROUNDS=3 STEPS=20 WARMUP=5 bash scripts/ab_env.sh - $SET || exit 1
ROUNDS=2 STEPS=1000 WARMUP=100 bash scripts/ab_env.sh - $SET || exit 1
