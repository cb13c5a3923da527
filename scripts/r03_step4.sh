#!/bin/bash
# Round-3 step 4: parity of the changed z kernel and the sparse NNGP path, bench 20 vs 1000,
# config-5 chain diagnostics, phylo under rocprofv3 with graph node counts (last).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s4}
mkdir -p $R/gpurun_out
cd $R
export HMSC_GRAPH_DEBUG=1
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_vignette2.py tests/test_gpu_spatial.py tests/test_gpu_spatial_large.py tests/test_gpu_post.py tests/test_gpu_determinism.py tests/test_gpu_multigpu.py -k "not posterior" -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 120 ./scripts/ubench_z > gpurun_out/${TAG}_ubz.log 2>&1 || { echo "ubench failed"; tail gpurun_out/${TAG}_ubz.log; exit 1; }
cat gpurun_out/${TAG}_ubz.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
cat gpurun_out/${TAG}_b20.json; grep hmsc gpurun_out/${TAG}_b20.err | head
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000.json 2> gpurun_out/${TAG}_b1000.err || { echo "bench1000 failed"; tail -20 gpurun_out/${TAG}_b1000.err; exit 1; }
cat gpurun_out/${TAG}_b1000.json
HMSC_ETA_FOUR_WAVES=1 timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000_eta4.json 2>/dev/null || { echo "bench eta4 failed"; exit 1; }
cat gpurun_out/${TAG}_b1000_eta4.json
timeout -k 10 200 python scripts/stamps_sweep.py > gpurun_out/${TAG}_stamps.log 2>&1 || { echo "stamps failed"; tail gpurun_out/${TAG}_stamps.log; exit 1; }
cat gpurun_out/${TAG}_stamps.log
timeout -k 10 600 python -u scripts/diag_spatial_chain.py 1000,1100,2100,5000 40 > gpurun_out/${TAG}_spchain.json 2> gpurun_out/${TAG}_spchain.err || { echo "spchain failed"; tail -20 gpurun_out/${TAG}_spchain.err; exit 1; }
cat gpurun_out/${TAG}_spchain.json
cd /tmp && export TMPDIR=/tmp
export HMSC_SEGV_DIAG=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_phyprof -o run -- python3 $R/bench.py --workload phylo --steps 100 --warmup 100 > $R/gpurun_out/${TAG}_phy.json 2> $R/gpurun_out/${TAG}_phy.err || { echo "phylo rocprof failed"; grep -a "hmsc\] captured" $R/gpurun_out/${TAG}_phy.err | head; grep -a "hmsc\]   #1[2-4]" $R/gpurun_out/${TAG}_phy.err; exit 1; }
cat $R/gpurun_out/${TAG}_phy.json; grep -a "hmsc\] captured" $R/gpurun_out/${TAG}_phy.err | head
