#!/bin/bash
# round 4 evidence A: the whole GPU suite, the driver-shaped lines, the default bench line
# and the kernel trace + stats of a 300-step bench run
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04_s3}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?
tail -2 gpurun_out/${TAG}_pytest_gpu.log
grep -E "FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_bench_steps20.json 2> gpurun_out/${TAG}_b20.err || { tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
cat gpurun_out/${TAG}_bench_steps20.json
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python $R/bench.py --steps 300 --warmup 30 --no-cpu > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err || { echo "rocprof failed"; tail -20 $R/gpurun_out/${TAG}_prof.err; exit 1; }
echo done
