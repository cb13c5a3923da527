#!/bin/bash
# quick parity + bench loop, then the kernel-trace A/B against the round-3 library
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/r04_quick.sh ${1:-r04_q} || exit 1
bash scripts/r04_ab3.sh || exit 1
