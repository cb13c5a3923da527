#!/bin/bash
# same-box A/B: the round-3 library (scripts/ab/lib_r3.so, built from c704414) against the
# current one, then the gamma2_bl / eta / side-chain clock stamps of both
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04_ab1}
cd $R
bash scripts/ab_bench.sh $TAG scripts/ab/lib_r3.so hmsc_amd/libhmsc_amd.so 3 || exit 1
for L in scripts/ab/lib_r3_stamps.so hmsc_amd/libhmsc_amd_stamps.so; do
  echo "== stamps $L"
  HMSC_AMD_LIB=$R/$L timeout -k 10 120 python scripts/stamps_sweep.py || exit 1
done
echo done
