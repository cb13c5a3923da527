#!/bin/bash
# dense-path check: the diagonal-block microbenchmark, the dense / phylogeny / GammaEta /
# spatial / handshake / config-3 GPU tests, then config 3 and config 5 Full bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04_dense}
cd $R
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/ubench_diag || exit 1
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_phylo.py tests/test_gpu_gamma_eta.py tests/test_gpu_handshake.py tests/test_gpu_config3.py tests/test_gpu_spatial.py > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_pytest.log
grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head -10
[ $rc -eq 0 ] || exit 1
for L in scripts/ab/lib_prev.so hmsc_amd/libhmsc_amd.so; do
  HMSC_AMD_LIB=$R/$L timeout -k 10 300 python bench.py --workload phylo --steps 100 --warmup 200 --no-cpu > gpurun_out/${TAG}_c3.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_c3.json'));print('$L config3', d['value'], d['roofline']['frac'], d['kernels_eager_events_us'])"
  HMSC_AMD_LIB=$R/$L timeout -k 10 300 python bench.py --workload spatial --method Full --steps 50 --warmup 10 --no-cpu > gpurun_out/${TAG}_c5.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_c5.json'));print('$L config5 full', d['value'])"
done
echo done
