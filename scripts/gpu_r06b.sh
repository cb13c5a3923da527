#!/bin/bash
# GPU-box helper (round 6): sharded-path tests, the bench line with its sharded leg, the
# 20-step line with the host timer, sharded timelines and the 20-sweep run's per-sweep timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06b}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_sharded_procs.py tests/test_gpu_determinism.py tests/test_gpu_capi_c.py tests/test_gpu_parity.py -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest.log | head -20
tail -2 gpurun_out/${TAG}_pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit 1;; esac
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print('main', d['value'], d['ms_per_step'], d['kernels_live_us'], 'sharded', d['sharded_chain']['value'], d['sharded_chain']['ms_per_step'])"
HMSC_DIAG_TIMING=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_b20.json').read().strip().splitlines()[-1]); print('b20', d['value'], d['ms_per_step'], 'sharded', d['sharded_chain']['value'], d['sharded_chain']['ms_per_step'])"
grep "run 20 sweeps" gpurun_out/${TAG}_b20.err | head -3
timeout -k 10 200 python -u scripts/run20_timeline.py > gpurun_out/${TAG}_run20.txt 2>&1 || { tail -20 gpurun_out/${TAG}_run20.txt; exit 1; }
grep "^run" gpurun_out/${TAG}_run20.txt
for v in "sharded_rec:--sharded --record" "sharded125_rec:--sharded --record --ns 125"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 200 python -u scripts/kt_timeline.py $a > gpurun_out/${TAG}_kt_$n.txt 2>&1 || { cat gpurun_out/${TAG}_kt_$n.txt; exit 1; }
  echo "== $n"; grep -v "version\|Hostname\|Librccl" gpurun_out/${TAG}_kt_$n.txt
done
