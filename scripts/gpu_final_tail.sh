#!/bin/bash
# the tail of gpu_final.sh (phylo rocprof pass and the config-3 / config-5 bench lines)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-final}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_phyprof -o run -- python3 $R/bench.py --workload phylo --steps 100 --warmup 100 --no-cpu > $R/gpurun_out/${TAG}_phyprof.json 2> $R/gpurun_out/${TAG}_phyprof.err || { echo "phylo rocprof failed"; tail -5 $R/gpurun_out/${TAG}_phyprof.err; exit 1; }
cd $R
timeout -k 10 300 python bench.py --workload phylo --steps 200 --warmup 200 > gpurun_out/${TAG}_config3.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --workload spatial --method GPP --steps 500 --warmup 50 > gpurun_out/${TAG}_config5_gpp.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --workload spatial --steps 20 --warmup 5 > gpurun_out/${TAG}_config5_full.json 2>/dev/null || exit 1
for f in config3 config5_gpp config5_full; do python -c "import json;d=json.load(open('gpurun_out/${TAG}_$f.json'));print('$f', d['value'], (d.get('cpu_baseline') or {}).get('value'))"; done
echo done
