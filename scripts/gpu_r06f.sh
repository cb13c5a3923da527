#!/bin/bash
# GPU-box helper (round 6): the sharded-vs-oracle test, then the 20-step line A/B'd over the
# bench's untimed clock warm-up (0.5 s vs 2 s).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_sharded_oracle.py -v --timeout 240 --timeout-method thread > gpurun_out/r06_n_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r06_n_pytest.log | cut -c1-120; tail -1 gpurun_out/r06_n_pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit 1;; esac
for r in 1 2 3 4; do
  for cw in 0.5 2.0; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-sharded-leg --clock-warmup-s $cw > gpurun_out/r06_cw_${cw}_$r.json 2>/dev/null || { echo "bench failed"; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r06_cw_${cw}_$r.json').read().strip().splitlines()[-1]); print('cw $cw', $r, d['value'], d['kernels_live_us'], d['clock_warmup_sweeps'])"
  done
done
