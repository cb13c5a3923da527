#!/bin/bash
# round 4, session 1: the whole GPU suite (new: config 3 as specified, default usage, handshake
# reports, NNGP ny=5000), then the driver-shaped bench line and the config 3 / 5 lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04_s1}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 60 ./scripts/ubench_rates > gpurun_out/${TAG}_rates.log 2>&1 && cat gpurun_out/${TAG}_rates.log
timeout -k 10 120 ./scripts/ubench_parts > gpurun_out/${TAG}_parts.log 2>&1 && cat gpurun_out/${TAG}_parts.log
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
grep -E "FAILED|Error|error" gpurun_out/${TAG}_pytest.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench20.json 2> gpurun_out/${TAG}_bench20.err || { tail -20 gpurun_out/${TAG}_bench20.err; exit 1; }
cat gpurun_out/${TAG}_bench20.json
timeout -k 10 300 python bench.py --workload spatial --method NNGP --steps 50 --warmup 10 --no-cpu > gpurun_out/${TAG}_config5_nngp_bench.json 2> gpurun_out/${TAG}_nngp.err || { tail -20 gpurun_out/${TAG}_nngp.err; exit 1; }
cat gpurun_out/${TAG}_config5_nngp_bench.json
timeout -k 10 300 python bench.py --workload phylo --steps 100 --warmup 200 --no-cpu > gpurun_out/${TAG}_config3_bench.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
cat gpurun_out/${TAG}_config3_bench.json
echo done
