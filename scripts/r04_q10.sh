#!/bin/bash
# quick parity loop + live timeline + graph stamps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/r04_quick.sh ${1:-r04_q10} || exit 1
timeout -k 10 200 python scripts/kt_timeline.py || exit 1
HMSC_AMD_LIB=$R/hmsc_amd/libhmsc_amd_stamps.so timeout -k 10 120 python scripts/stamps_sweep.py --graph 2>&1 | grep -E "gamma2_bl|tail|side" || exit 1
