#!/bin/bash
# GPU-box helper: live-timer sweep timelines -- sharded (one-rank RCCL) without and with the
# record, unsharded with it, and the ns = 125 sharded proxy.  usage: gpu_kt3.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
mkdir -p $R/gpurun_out
cd $R
for v in "sharded:--sharded" "sharded_rec:--sharded --record" "unsharded_rec:--record" "sharded125_rec:--sharded --record --ns 125" "unsharded125_rec:--record --ns 125"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 200 python -u scripts/kt_timeline.py $a > gpurun_out/${TAG}_kt_$n.txt 2>&1 || { cat gpurun_out/${TAG}_kt_$n.txt; exit 1; }
  echo "== $n"; grep -v "version\|Hostname\|Librccl" gpurun_out/${TAG}_kt_$n.txt
done
