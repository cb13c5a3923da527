#!/bin/bash
# same-box A/B/C of three library builds: alternating 1000-step bench runs
# usage: ab_bench3.sh TAG LIB_A LIB_B LIB_C [ROUNDS]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; N=${5:-3}
mkdir -p $R/gpurun_out
cd $R
for i in $(seq 1 $N); do
for L in A B C; do
  case $L in A) LIB=$2;; B) LIB=$3;; C) LIB=$4;; esac
  HMSC_AMD_LIB=$R/$LIB timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${TAG}_${L}_$i.json 2> gpurun_out/${TAG}_${L}_$i.err || { echo "bench $L failed"; tail -20 gpurun_out/${TAG}_${L}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_${L}_$i.json'));print('$L', d['value'], d.get('kernels_live_us'))"
done
done
