#!/bin/bash
# GPU-box helper: the whole -m gpu suite (names in the log), then the 1000-step and the
# driver-shaped 20-step bench lines (no CPU baseline).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-check}
mkdir -p $R/gpurun_out
cd $R
# (no -x: every failure is listed; a failing test does not stop the bench lines, but a crash,
# a fault or the time limit does -- exit 124 / 134 / 137 / 139 end the script)
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest.log | head -40
tail -2 gpurun_out/${TAG}_pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit 1;; esac
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
cat gpurun_out/${TAG}_b20.json
timeout -k 10 120 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/${TAG}_g2.json 2> gpurun_out/${TAG}_g2.err; echo "gpus=2 on one GPU: rc=$? $(cat gpurun_out/${TAG}_g2.err)"
