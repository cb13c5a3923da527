#!/bin/bash
# round 4 quick loop: the config-4 parity / full-size / determinism tests, then the driver-shaped
# 20-step line and a 1000-step line (no CPU baseline)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04_q}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_determinism.py tests/test_gpu_nf.py tests/test_gpu_kernel_timing.py ${EXTRA_TESTS} > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_pytest.log
grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head -10
[ $rc -eq 0 ] || exit 1
for n in 20 1000; do
  timeout -k 10 300 python bench.py --steps $n --warmup 5 --no-cpu > gpurun_out/${TAG}_bench$n.json 2> gpurun_out/${TAG}_bench$n.err || { tail -20 gpurun_out/${TAG}_bench$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench$n.json'));print($n, d['value'], d['ms_per_step'], d['kernels_live_us'])"
done
echo done
