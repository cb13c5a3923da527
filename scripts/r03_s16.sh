#!/bin/bash
# Flag-ordered side chain (no fork edge): the whole GPU suite, bench 1000 and 20, a trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s16}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread -k "graph or sweep" > gpurun_out/${TAG}_pytest0.log 2>&1 || { echo "pytest0 failed"; tail -40 gpurun_out/${TAG}_pytest0.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest0.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b1000.json 2> gpurun_out/${TAG}_b1000.err || { echo "bench1000 failed"; tail -20 gpurun_out/${TAG}_b1000.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_b1000.json'));print('steps1000', d['value'], d['kernels_live_us'], d['kernels_eager_events_us'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_b20.json'));print('steps20', d['value'], d['kernels_live_us'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --steps 300 --warmup 100 --no-cpu --ess-samples 1000 > $R/gpurun_out/${TAG}_prof.json 2> $R/gpurun_out/${TAG}_prof.err || { echo "rocprof failed"; tail -5 $R/gpurun_out/${TAG}_prof.err; exit 1; }
echo prof ok
