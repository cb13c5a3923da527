#!/bin/bash
# A/B of the BetaLambda tail's tile publication (write-through stores vs plain + one L2
# write-back per workgroup): graph stamps and 1000-step bench lines, alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for m in 0 1; do
  echo "== HMSC_TAIL_PUB=$m"
  HMSC_TAIL_PUB=$m HMSC_AMD_LIB=$R/hmsc_amd/libhmsc_amd_stamps.so timeout -k 10 120 python scripts/stamps_sweep.py --graph 2>&1 | grep -E "gamma2_bl|tail" || exit 1
done
for i in 1 2; do for m in 0 1; do
  HMSC_TAIL_PUB=$m timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/pub_${m}_$i.json 2> gpurun_out/pub_${m}_$i.err || { tail -5 gpurun_out/pub_${m}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/pub_${m}_$i.json'));print('pub $m', d['value'], d.get('kernels_live_us'))"
done; done
echo done
