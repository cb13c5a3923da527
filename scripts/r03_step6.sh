#!/bin/bash
# Round-3 step 6: config-5 chain tests, the fixed cost of one run call, then configs 3 and 5
# with their CPU baselines (numpy restatement), and config 3 under rocprofv3 with graphs
# capped at 256 nodes (the profiler-aware cap).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s6}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_config5_chain.py tests/test_gpu_spatial_large.py -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -4 gpurun_out/${TAG}_pytest.log
HMSC_DIAG_TIMING=1 timeout -k 10 300 python -u scripts/run_overhead.py > gpurun_out/${TAG}_overhead.log 2>&1 || { echo "overhead failed"; tail -20 gpurun_out/${TAG}_overhead.log; exit 1; }
cat gpurun_out/${TAG}_overhead.log
timeout -k 10 400 python -u bench.py --workload phylo --steps 200 --warmup 200 > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { echo "config3 failed"; tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
cat gpurun_out/${TAG}_c3.json
for M in Full NNGP GPP; do
timeout -k 10 900 python -u bench.py --workload spatial --method $M --steps 100 --warmup 20 > gpurun_out/${TAG}_c5_$M.json 2> gpurun_out/${TAG}_c5_$M.err || { echo "config5 $M failed"; tail -20 gpurun_out/${TAG}_c5_$M.err; exit 1; }
cat gpurun_out/${TAG}_c5_$M.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_phyprof -o run -- python3 $R/bench.py --workload phylo --steps 100 --warmup 100 --no-cpu > $R/gpurun_out/${TAG}_phyprof.json 2> $R/gpurun_out/${TAG}_phyprof.err || { echo "phylo rocprof failed"; tail -5 $R/gpurun_out/${TAG}_phyprof.err; exit 1; }
echo "phylo under rocprofv3 with the profiler cap: ok"; cat $R/gpurun_out/${TAG}_phyprof.json
