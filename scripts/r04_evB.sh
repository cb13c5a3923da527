#!/bin/bash
# round 4 evidence B: PMC passes over the synthetic sweep (z, eta, gamma2_bl, side chain),
# a kernel trace restricted to the main-queue kernels, and the config 3 / 5 lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04_s3}
cd $R
bash scripts/pmc_z.sh ${TAG}_pmc "z_wave|eta_fused|gamma2_bl|side_chain|slab_pack" || exit 1
python scripts/pmc_summary.py gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_pmc.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "z_wave|eta_fused|gamma2_bl|slab_pack" --output-format csv -d $R/gpurun_out/${TAG}_profmain -o run -- python $R/bench.py --steps 300 --warmup 30 --no-cpu > $R/gpurun_out/${TAG}_profmain_bench.json 2> $R/gpurun_out/${TAG}_profmain.err || { echo "rocprof failed"; tail -20 $R/gpurun_out/${TAG}_profmain.err; exit 1; }
cd $R
timeout -k 10 300 python bench.py --workload phylo --steps 100 --warmup 200 --no-cpu > gpurun_out/${TAG}_config3_bench.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
timeout -k 10 300 python bench.py --workload spatial --method Full --steps 50 --warmup 10 --no-cpu > gpurun_out/${TAG}_config5_full_bench.json 2> gpurun_out/${TAG}_c5f.err || { tail -20 gpurun_out/${TAG}_c5f.err; exit 1; }
timeout -k 10 300 python bench.py --workload spatial --method GPP --steps 200 --warmup 20 --no-cpu > gpurun_out/${TAG}_config5_gpp_bench.json 2> gpurun_out/${TAG}_c5g.err || { tail -20 gpurun_out/${TAG}_c5g.err; exit 1; }
timeout -k 10 300 python bench.py --workload spatial --method NNGP --steps 50 --warmup 10 --no-cpu > gpurun_out/${TAG}_config5_nngp_bench.json 2> gpurun_out/${TAG}_c5n.err || { tail -20 gpurun_out/${TAG}_c5n.err; exit 1; }
for f in config3 config5_full config5_gpp config5_nngp; do python -c "import json;d=json.load(open('gpurun_out/${TAG}_${f}_bench.json'));print('$f', d['value'], d.get('start'))"; done
echo done
