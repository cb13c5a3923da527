#!/bin/bash
# GPU-box helper: sharded-chain changes -- their parity tests, the bench line with its sharded
# leg, the sharded timelines, a kernel trace, and the 20-step line's host timing breakdown.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-shard2}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_sharded_procs.py tests/test_gpu_determinism.py tests/test_gpu_capi_c.py -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest.log | head -20
tail -2 gpurun_out/${TAG}_pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit 1;; esac
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]); print('main', d['value'], d['ms_per_step'], 'sharded', d['sharded_chain'])"
HMSC_DIAG_TIMING=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-sharded-leg > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_b20.json').read()); print('b20', d['value'], d['ms_per_step'])"
grep -i "diag\|enqueue\|run " gpurun_out/${TAG}_b20.err | tail -12
timeout -k 10 200 python -u scripts/kt_timeline.py --record --sharded > gpurun_out/${TAG}_kt_sharded.txt 2>&1 || { cat gpurun_out/${TAG}_kt_sharded.txt; exit 1; }
timeout -k 10 200 python -u scripts/kt_timeline.py --record --sharded --ns 125 > gpurun_out/${TAG}_kt_sharded125.txt 2>&1 || { cat gpurun_out/${TAG}_kt_sharded125.txt; exit 1; }
for f in kt_sharded kt_sharded125; do echo "== $f"; grep -v "version\|Hostname\|Librccl" gpurun_out/${TAG}_$f.txt; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_trace -o run -- python $R/scripts/trace_sharded.py > $R/gpurun_out/${TAG}_trace.log 2>&1 || { echo "trace failed"; tail -20 $R/gpurun_out/${TAG}_trace.log; exit 1; }
cd $R
f=$(find gpurun_out/${TAG}_trace -name '*kernel_trace.csv' | head -1)
python scripts/trace_view.py $f gamma2_bl_kernel 2 150 > gpurun_out/${TAG}_trace_view.txt 2>&1
cat gpurun_out/${TAG}_trace_view.txt
