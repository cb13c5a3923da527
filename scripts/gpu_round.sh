#!/bin/bash
# One GPU round: parity tests, PMC passes of the dominant kernels, bench (reading that PMC
# summary for roofline.traffic), rocprofv3 kernel-trace stats of the same bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-run}
STEPS=${STEPS:-1000}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
bash scripts/pmc_z.sh ${TAG}_pmc "z_wave|eta_fused|beta_lambda|gammav_wave" || exit 1
python scripts/pmc_summary.py gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_pmc.json || exit 1
timeout -k 10 600 python bench.py --steps $STEPS --warmup 100 --pmc-json gpurun_out/${TAG}_pmc.json > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python $R/bench.py --steps $STEPS --warmup 100 --no-cpu --pmc-json $R/gpurun_out/${TAG}_pmc.json > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err || { echo "rocprof failed"; tail -20 $R/gpurun_out/${TAG}_prof.err; exit 1; }
cat $R/gpurun_out/${TAG}_prof_bench.json
echo done
