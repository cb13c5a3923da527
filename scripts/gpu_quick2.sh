#!/bin/bash
# GPU-box helper: the GPU parity suite, one bench line and a rocprofv3 kernel-stats pass of a
# short bench (no CPU baseline, no PMC).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-q2}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --steps ${STEPS:-1000} --warmup 100 --no-cpu > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python $R/bench.py --steps 300 --warmup 30 --no-cpu > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err || { echo "rocprof failed"; tail -20 $R/gpurun_out/${TAG}_prof.err; exit 1; }
echo done
