#!/bin/bash
# GPU-box helper (round 6): the GPU suite, a same-box A/B of two library builds, the sharded
# diagnostic.  usage: gpu_r06.sh TAG LIB_A LIB_B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; A=$2; B=$3
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest.log | head -30
tail -2 gpurun_out/${TAG}_pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit 1;; esac
ROUNDS=2 bash scripts/ab_lib.sh $A $B || exit 1
timeout -k 10 400 python -u scripts/sharded_diag.py > gpurun_out/${TAG}_diag.log 2> gpurun_out/${TAG}_diag.err || { tail -20 gpurun_out/${TAG}_diag.err; exit 1; }
grep -v "version\|Hostname\|Librccl" gpurun_out/${TAG}_diag.log
