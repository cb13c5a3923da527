#!/bin/bash
# quick parity loop + graph stamps + two 1000-step lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/r04_quick.sh ${1:-r04_q8} || exit 1
HMSC_AMD_LIB=$R/hmsc_amd/libhmsc_amd_stamps.so timeout -k 10 120 python scripts/stamps_sweep.py --graph 2>&1 | grep -E "gamma2_bl|tail|side" || exit 1
timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --no-cpu > gpurun_out/${1:-r04_q8}_b2.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/${1:-r04_q8}_b2.json'));print('1000 again', d['value'], d.get('kernels_live_us'))"
