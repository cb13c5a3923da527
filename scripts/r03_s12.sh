#!/bin/bash
# Fused Gamma2 + BetaLambda launch: the whole GPU suite, bench 20 vs 1000, run overhead.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s12}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
cat gpurun_out/${TAG}_b20.json
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000.json 2> gpurun_out/${TAG}_b1000.err || { echo "bench1000 failed"; tail -20 gpurun_out/${TAG}_b1000.err; exit 1; }
cat gpurun_out/${TAG}_b1000.json
HMSC_DIAG_TIMING=1 timeout -k 10 300 python -u scripts/run_overhead.py > gpurun_out/${TAG}_overhead.log 2>&1 || { echo "overhead failed"; tail -20 gpurun_out/${TAG}_overhead.log; exit 1; }
grep "S=20\|S=1000\|run 20 \|run 1000 " gpurun_out/${TAG}_overhead.log
