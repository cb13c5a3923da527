#!/bin/bash
# the driver-shaped 20-step line with the run's host-side breakdown (HMSC_DIAG_TIMING)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for i in 1 2; do
HMSC_DIAG_TIMING=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/b20_$i.json 2> gpurun_out/b20_$i.err || { tail -20 gpurun_out/b20_$i.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b20_$i.json'));print('20', d['value'], d['ms_per_step'])"
grep "\[hmsc\] run" gpurun_out/b20_$i.err | tail -6
done
