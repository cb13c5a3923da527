#!/bin/bash
# where the fused Gamma2 + BetaLambda launch's tail spends its time (stamps library) + live timeline
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r04_tail.log
: > $out
timeout -k 10 120 python -u scripts/stamps_sweep.py --graph --blocks >> $out 2>&1 &&
timeout -k 10 120 python -u scripts/kt_timeline.py --record >> $out 2>&1
