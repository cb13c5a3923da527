#!/bin/bash
# GPU-box helper (round 6): the record-copy equivalence test, a runtime trace of the
# driver-shaped 20-step line (scripts/rt_view.py), then the final evidence's part B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06_s2}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_record_copy.py -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_rc_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_rc_pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit 1;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --runtime-trace --output-format csv -d $R/gpurun_out/${TAG}_rt -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --no-sharded-leg > $R/gpurun_out/${TAG}_rt_bench.json 2> $R/gpurun_out/${TAG}_rt.err || { echo "runtime trace failed"; tail -5 $R/gpurun_out/${TAG}_rt.err; exit 1; }
cd $R
python scripts/rt_view.py gpurun_out/${TAG}_rt > gpurun_out/${TAG}_rt_view.txt 2>&1; tail -4 gpurun_out/${TAG}_rt_view.txt
PART=B bash scripts/gpu_final.sh $TAG
