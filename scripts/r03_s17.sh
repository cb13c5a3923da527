#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s17}
mkdir -p $R/gpurun_out
cd $R
for NG in 1 0; do
HMSC_NO_GRAPH=$NG timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000_ng$NG.json 2> gpurun_out/${TAG}_b1000_ng$NG.err || { echo "bench1000 failed"; tail -20 gpurun_out/${TAG}_b1000_ng$NG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_b1000_ng$NG.json'));print('no_graph=$NG', d['value'], d['kernels_live_us'])"
HMSC_NO_GRAPH=$NG timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20_ng$NG.json 2> gpurun_out/${TAG}_b20_ng$NG.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20_ng$NG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_b20_ng$NG.json'));print('steps20 no_graph=$NG', d['value'])"
done
