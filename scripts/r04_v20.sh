#!/bin/bash
# 20-step driver-shaped lines and the 20-sweep run timeline under environment variants
# usage: r04_v20.sh TAG "VAR=1" ...   ("-" = no variable)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  e=$v; [ "$e" = "-" ] && e=""
  echo "== $v" >> gpurun_out/${TAG}_t20.log
  env $e timeout -k 10 120 python -u scripts/run20_timeline.py 20 >> gpurun_out/${TAG}_t20.log 2>&1 || exit 1
  for i in 1 2; do
    env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_b20.json'));print('$v', d['value'], d.get('kernels_live_us'))"
  done
done
