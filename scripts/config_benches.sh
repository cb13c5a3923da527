#!/bin/bash
# Config 3 / config 5 bench lines with their CPU baselines (numpy restatement), into gpurun_out/cfg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/cfg
cd $R
timeout -k 10 300 python -u bench.py --workload phylo --steps 200 --warmup 50 > gpurun_out/cfg/config3.json 2> gpurun_out/cfg/config3.err || { echo "config3 failed"; tail -5 gpurun_out/cfg/config3.err; exit 1; }
for m in GPP NNGP Full; do
  timeout -k 10 600 python -u bench.py --workload spatial --method $m --steps 200 --warmup 50 > gpurun_out/cfg/config5_$m.json 2> gpurun_out/cfg/config5_$m.err || { echo "config5 $m failed"; tail -5 gpurun_out/cfg/config5_$m.err; exit 1; }
done
echo configs done
