#!/bin/bash
# Eta tile staging + per-sample copied flags: parity tests, bench 20 vs 1000, run overhead,
# and a kernel trace of the bench for the per-sweep timeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s11}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_nf.py tests/test_gpu_kernel_timing.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
cat gpurun_out/${TAG}_b20.json
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000.json 2> gpurun_out/${TAG}_b1000.err || { echo "bench1000 failed"; tail -20 gpurun_out/${TAG}_b1000.err; exit 1; }
cat gpurun_out/${TAG}_b1000.json
HMSC_DIAG_TIMING=1 timeout -k 10 300 python -u scripts/run_overhead.py > gpurun_out/${TAG}_overhead.log 2>&1 || { echo "overhead failed"; tail -20 gpurun_out/${TAG}_overhead.log; exit 1; }
grep "S=20\|S=1000" gpurun_out/${TAG}_overhead.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --steps 400 --warmup 100 --no-cpu --ess-samples 1000 > $R/gpurun_out/${TAG}_prof.json 2> $R/gpurun_out/${TAG}_prof.err || { echo "rocprof failed"; tail -5 $R/gpurun_out/${TAG}_prof.err; exit 1; }
echo prof ok
