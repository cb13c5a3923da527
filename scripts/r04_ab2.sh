#!/bin/bash
# gamma2_bl clock stamps inside graph replays: round-3 library against the current one
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for rep in 1 2; do
for L in scripts/ab/lib_r3_stamps.so hmsc_amd/libhmsc_amd_stamps.so; do
  echo "== graph stamps $L"
  HMSC_AMD_LIB=$R/$L timeout -k 10 120 python scripts/stamps_sweep.py --graph 2>&1 | grep -v "^\[hmsc\]" || exit 1
done
done
echo done
