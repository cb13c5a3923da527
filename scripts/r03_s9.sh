#!/bin/bash
# z-kernel layout A/B: the LDS-transposed draw (z_wave_kernel) vs the matrix-core-layout draw
# (z_reg_kernel) without and with the register prefetch of the next tile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s9}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 120 ./scripts/ubench_z > gpurun_out/${TAG}_wave.log 2>&1 || { echo "ubench wave failed"; tail gpurun_out/${TAG}_wave.log; exit 1; }
cat gpurun_out/${TAG}_wave.log
timeout -k 10 120 ./scripts/ubench_z r > gpurun_out/${TAG}_reg0.log 2>&1 || { echo "ubench reg0 failed"; tail gpurun_out/${TAG}_reg0.log; exit 1; }
cat gpurun_out/${TAG}_reg0.log
timeout -k 10 120 ./scripts/ubench_zr1 r > gpurun_out/${TAG}_reg1.log 2>&1 || { echo "ubench reg1 failed"; tail gpurun_out/${TAG}_reg1.log; exit 1; }
cat gpurun_out/${TAG}_reg1.log
