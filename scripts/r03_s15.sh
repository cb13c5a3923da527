#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s15}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 200 python scripts/stamps_sweep.py > gpurun_out/${TAG}_stamps.log 2>&1 || { echo "stamps failed"; tail gpurun_out/${TAG}_stamps.log; exit 1; }
head -1 gpurun_out/${TAG}_stamps.log; grep "beta_lambda\|gamma2_final" gpurun_out/${TAG}_stamps.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_vignette2.py tests/test_gpu_predict.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for V in 0 1; do
HMSC_NO_G2BL_FUSION=$V timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000_nf$V.json 2> gpurun_out/${TAG}_b1000_nf$V.err || { echo "bench1000 failed"; tail -20 gpurun_out/${TAG}_b1000_nf$V.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_b1000_nf$V.json'));print('no_fusion=$V', d['value'], d['kernels_live_us'], d['kernels_eager_events_us'])"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_b20.json'));print('steps20', d['value'], d['kernels_live_us'])"
HMSC_DIAG_TIMING=1 timeout -k 10 300 python -u scripts/run_overhead.py > gpurun_out/${TAG}_overhead.log 2>&1 || { echo "overhead failed"; tail -20 gpurun_out/${TAG}_overhead.log; exit 1; }
grep "S=20\|run 20 " gpurun_out/${TAG}_overhead.log
