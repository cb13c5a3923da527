#!/bin/bash
# persistent unpack pool: record tests, then bench 1000 / 20 steps (x3 for the 20-step line)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s18}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_posterior.py > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000.json 2> gpurun_out/${TAG}_b1000.err || { echo "bench1000 failed"; tail -20 gpurun_out/${TAG}_b1000.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_b1000.json'));print('1000', d['value'])"
for i in 1 2 3; do
HMSC_DIAG_TIMING=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20_$i.json 2> gpurun_out/${TAG}_b20_$i.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20_$i.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_b20_$i.json'));print('steps20', d['value'])"
grep "run 20 sweeps" gpurun_out/${TAG}_b20_$i.err | tail -2
done
