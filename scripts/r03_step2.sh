#!/bin/bash
# Round-3 step 2: driver-style bench line (graphs prebuilt), config-2 tests, config-5
# diagnostics, then the phylo workload under rocprofv3 (the graph node cap, last).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s2}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
cat gpurun_out/${TAG}_b20.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_vignette2.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
timeout -k 10 600 python -u scripts/diag_config5.py --np 2500 --ny 5000 --sweeps 300 > gpurun_out/${TAG}_c5diag.json 2> gpurun_out/${TAG}_c5diag.err || { echo "diag failed"; tail -20 gpurun_out/${TAG}_c5diag.err; exit 1; }
tail -1 gpurun_out/${TAG}_c5diag.json
cd /tmp && export TMPDIR=/tmp
export HMSC_SEGV_DIAG=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_phyprof -o run -- python3 $R/bench.py --workload phylo --steps 100 --warmup 100 > $R/gpurun_out/${TAG}_phy.json 2> $R/gpurun_out/${TAG}_phy.err || { echo "phylo rocprof failed"; grep -a "hmsc\]" $R/gpurun_out/${TAG}_phy.err | head -30; exit 1; }
cat $R/gpurun_out/${TAG}_phy.json
