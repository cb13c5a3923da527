#!/bin/bash
# kernel trace of both libraries (round 3 / current) on one box: per-kernel durations
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for L in A B; do
  LIB=scripts/ab/lib_r3.so; [ $L = B ] && LIB=hmsc_amd/libhmsc_amd.so
  HMSC_AMD_LIB=$R/$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab3_$L -o run -- python $R/bench.py --steps 300 --warmup 30 --no-cpu > $R/gpurun_out/ab3_${L}_bench.json 2> $R/gpurun_out/ab3_$L.err || { echo "rocprof $L failed"; tail -20 $R/gpurun_out/ab3_$L.err; exit 1; }
  python -c "import json;d=json.load(open('$R/gpurun_out/ab3_${L}_bench.json'));print('$L', d['value'], d.get('kernels_live_us'))"
done
echo done
