#!/bin/bash
# graph-mode clock stamps of the current library (gamma2_bl, its tail, the side chain)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for rep in 1 2; do
  HMSC_AMD_LIB=$R/hmsc_amd/libhmsc_amd_stamps.so timeout -k 10 120 python scripts/stamps_sweep.py --graph --blocks 2>&1 | grep -v "^\[hmsc\]" || exit 1
done
echo done
