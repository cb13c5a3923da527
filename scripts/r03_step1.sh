#!/bin/bash
# Round-3 step 1 on the GPU box: the driver's bench line (--steps 20 --warmup 5) with the
# graphs prebuilt, a 1000-step line for comparison, then the phylo workload under
# rocprofv3 --kernel-trace with the fault diagnostics on (last: it crashed in round 2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s1}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
cat gpurun_out/${TAG}_b20.json
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000.json 2> gpurun_out/${TAG}_b1000.err || { echo "bench1000 failed"; tail -20 gpurun_out/${TAG}_b1000.err; exit 1; }
cat gpurun_out/${TAG}_b1000.json
cd /tmp && export TMPDIR=/tmp
export HMSC_SEGV_DIAG=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_phyprof -o run -- python3 $R/bench.py --workload phylo --steps 100 --warmup 100 > $R/gpurun_out/${TAG}_phy.json 2> $R/gpurun_out/${TAG}_phy.err || { echo "phylo rocprof failed"; grep -a "hmsc\]" $R/gpurun_out/${TAG}_phy.err | head -80; exit 1; }
cat $R/gpurun_out/${TAG}_phy.json
