#!/bin/bash
# the next panel step inside the trailing update (opt-in HMSC_CHOL_PANEL_FUSION=1): dense /
# spatial / phylo / GammaEta parity with it on, same-box config 3 / 5 on and off, chol trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s33}
mkdir -p $R/gpurun_out
cd $R
HMSC_CHOL_PANEL_FUSION=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dense.py tests/test_gpu_spatial.py tests/test_gpu_phylo.py tests/test_gpu_gamma_eta.py tests/test_gpu_spatial_large.py > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" gpurun_out/${TAG}_pytest.log | head; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for PF in 1 0; do
  if [ $PF = 1 ]; then export HMSC_CHOL_PANEL_FUSION=1; else unset HMSC_CHOL_PANEL_FUSION; fi
  timeout -k 10 300 python bench.py --workload spatial --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_c5_pf$PF.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_c5_pf$PF.json'));print('config5 full panel_fusion=$PF', d['value'], d.get('kernels_eager_events_us'))"
  timeout -k 10 300 python bench.py --workload phylo --steps 100 --warmup 200 --no-cpu > gpurun_out/${TAG}_c3_pf$PF.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_c3_pf$PF.json'));print('config3 panel_fusion=$PF', d['value'], d.get('kernels_eager_events_us'))"
done
export HMSC_CHOL_PANEL_FUSION=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_chol -o run -- python $R/scripts/chol_bench.py 5000 3 > $R/gpurun_out/${TAG}_chol.log 2>&1 || { echo "chol profile failed"; exit 1; }
grep residual $R/gpurun_out/${TAG}_chol.log
head -6 $R/gpurun_out/${TAG}_chol/run_kernel_stats.csv | cut -c1-120
