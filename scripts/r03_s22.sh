#!/bin/bash
# spatial GammaEta blocked path tests + pipelined Eta stream: parity, bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s21}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_determinism.py tests/test_gpu_posterior.py tests/test_gpu_predict.py > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/${TAG}_pytest.log | head -20; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000.json 2> gpurun_out/${TAG}_b1000.err || { echo "bench1000 failed"; tail -20 gpurun_out/${TAG}_b1000.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_b1000.json'));print('1000', d['value'], d.get('kernels_live_us'))"
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20_$i.json 2> gpurun_out/${TAG}_b20_$i.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20_$i.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_b20_$i.json'));print('steps20', d['value'])"
done
timeout -k 10 200 python scripts/stamps_sweep.py > gpurun_out/${TAG}_stamps.txt 2>&1 && head -1 gpurun_out/${TAG}_stamps.txt
