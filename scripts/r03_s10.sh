#!/bin/bash
# Power-of-two graph replays + record-page pretouch: graph/record parity tests, the new
# conditional-prediction oracle test, bench 20 vs 1000 steps, the fixed cost of a run call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s10}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 120 ./scripts/ubench_parts > gpurun_out/${TAG}_parts.log 2>&1 || { echo "ubench_parts failed"; tail gpurun_out/${TAG}_parts.log; exit 1; }
cat gpurun_out/${TAG}_parts.log
timeout -k 10 120 ./scripts/ubench_z > gpurun_out/${TAG}_ubz.log 2>&1 || { echo "ubench_z failed"; tail gpurun_out/${TAG}_ubz.log; exit 1; }
head -12 gpurun_out/${TAG}_ubz.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_vignette2.py tests/test_gpu_predict.py tests/test_gpu_determinism.py tests/test_gpu_capi_c.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
cat gpurun_out/${TAG}_b20.json
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000.json 2> gpurun_out/${TAG}_b1000.err || { echo "bench1000 failed"; tail -20 gpurun_out/${TAG}_b1000.err; exit 1; }
cat gpurun_out/${TAG}_b1000.json
HMSC_DIAG_TIMING=1 timeout -k 10 300 python -u scripts/run_overhead.py > gpurun_out/${TAG}_overhead.log 2>&1 || { echo "overhead failed"; tail -20 gpurun_out/${TAG}_overhead.log; exit 1; }
cat gpurun_out/${TAG}_overhead.log
