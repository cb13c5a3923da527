#!/bin/bash
# recorded vs unrecorded sweeps: live timelines and the kernel traces of both
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
echo "== unrecorded"; timeout -k 10 200 python scripts/kt_timeline.py || exit 1
echo "== recorded"; timeout -k 10 200 python scripts/kt_timeline.py --record || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trnr -o run -- python $R/scripts/kt_timeline.py > /dev/null 2>&1 || exit 1
cd $R && python scripts/trace_timeline.py gpurun_out/trnr/run_kernel_trace.csv 100 200 | head -10
