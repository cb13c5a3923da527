#!/bin/bash
# live per-sweep timeline and 1000-step bench under environment variants of one library build
# usage: r04_variants.sh TAG "VAR=1" "VAR2=1" ...   ("-" = no variable)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  e=$v; [ "$e" = "-" ] && e=""
  echo "== $v" >> gpurun_out/${TAG}_kt.log
  env $e timeout -k 10 120 python -u scripts/kt_timeline.py --record >> gpurun_out/${TAG}_kt.log 2>&1 || exit 1
  env $e timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_b.json 2> gpurun_out/${TAG}_b.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_b.json'));print('$v', d['value'], d.get('kernels_live_us'))"
done
