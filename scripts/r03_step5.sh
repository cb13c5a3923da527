#!/bin/bash
# Round-3 step 5: GPU tests on the changed side chain / delta draws, bench 20 vs 1000 with the
# clock-ramp warm-up, Eta variants, stamps, config-5 long chains, then rocprofv3 experiments on
# the graph-launch crash (graphs off for phylo; config 4 at 256 and 512 graph nodes, last).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s5}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_sharded.py tests/test_gpu_nf.py tests/test_gpu_kernel_timing.py tests/test_gpu_determinism.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
cat gpurun_out/${TAG}_b20.json
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000.json 2> gpurun_out/${TAG}_b1000.err || { echo "bench1000 failed"; tail -20 gpurun_out/${TAG}_b1000.err; exit 1; }
cat gpurun_out/${TAG}_b1000.json
HMSC_ETA_DB=1 timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000_db1.json 2>/dev/null || { echo "bench db1 failed"; exit 1; }
cat gpurun_out/${TAG}_b1000_db1.json
timeout -k 10 200 python scripts/stamps_sweep.py > gpurun_out/${TAG}_stamps.log 2>&1 || { echo "stamps failed"; tail gpurun_out/${TAG}_stamps.log; exit 1; }
cat gpurun_out/${TAG}_stamps.log
timeout -k 10 400 python -u scripts/diag_config5_long.py 5000 400 > gpurun_out/${TAG}_c5long.json 2> gpurun_out/${TAG}_c5long.err || { echo "c5long failed"; tail -20 gpurun_out/${TAG}_c5long.err; exit 1; }
tail -1 gpurun_out/${TAG}_c5long.json
cd /tmp && export TMPDIR=/tmp
HMSC_NO_GRAPH=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_phyprof -o run -- python3 $R/bench.py --workload phylo --steps 50 --warmup 100 --no-cpu > $R/gpurun_out/${TAG}_phy_nograph.json 2> $R/gpurun_out/${TAG}_phy_nograph.err || { echo "phylo rocprof (no graphs) failed"; tail -5 $R/gpurun_out/${TAG}_phy_nograph.err; exit 1; }
echo "phylo under rocprofv3 without graphs: ok"; cat $R/gpurun_out/${TAG}_phy_nograph.json
HMSC_GRAPH_DEBUG=1 HMSC_GRAPH_SWEEPS=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_g32prof -o run -- python3 $R/bench.py --steps 200 --warmup 100 --no-cpu --ess-samples 1000 > $R/gpurun_out/${TAG}_g32.json 2> $R/gpurun_out/${TAG}_g32.err || { echo "config4 rocprof at 32 sweeps/graph failed"; grep -a "hmsc\]" $R/gpurun_out/${TAG}_g32.err | head; exit 1; }
echo "config 4 under rocprofv3 with 32-sweep graphs: ok"; grep -a "hmsc\] captured" $R/gpurun_out/${TAG}_g32.err | head -3
HMSC_GRAPH_DEBUG=1 HMSC_GRAPH_SWEEPS=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_g64prof -o run -- python3 $R/bench.py --steps 200 --warmup 100 --no-cpu --ess-samples 1000 > $R/gpurun_out/${TAG}_g64.json 2> $R/gpurun_out/${TAG}_g64.err || { echo "config4 rocprof at 64 sweeps/graph failed"; grep -a "hmsc\]" $R/gpurun_out/${TAG}_g64.err | head; exit 1; }
echo "config 4 under rocprofv3 with 64-sweep graphs: ok"; grep -a "hmsc\] captured" $R/gpurun_out/${TAG}_g64.err | head -3
