#!/bin/bash
# Round-end evidence on one GPU: the full GPU parity suite (test names in the log), smoke(),
# PMC passes of the dominant kernels, the headline bench reading that PMC summary, a
# rocprofv3 kernel-trace --stats pass of the same bench, and the config-3 / config-5 lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-final}
PART=${PART:-all}   # A: tests, PMC, config-4 lines and profile; B: dense / config-3 / config-5
mkdir -p $R/gpurun_out
cd $R
if [ "$PART" != "B" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
bash scripts/pmc_z.sh ${TAG}_pmc "z_wave|eta_fused|beta_lambda|side_chain" || exit 1
python scripts/pmc_summary.py gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_pmc.json || exit 1
timeout -k 10 600 python bench.py --steps 1000 --warmup 100 --pmc-json gpurun_out/${TAG}_pmc.json > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --pmc-json gpurun_out/${TAG}_pmc.json --no-cpu > gpurun_out/${TAG}_b20.json 2> gpurun_out/${TAG}_b20.err || { echo "bench20 failed"; tail -20 gpurun_out/${TAG}_b20.err; exit 1; }
cat gpurun_out/${TAG}_b20.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python $R/bench.py --steps 1000 --warmup 100 --no-cpu --no-sharded-leg --pmc-json $R/gpurun_out/${TAG}_pmc.json > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err || { echo "rocprof failed"; tail -20 $R/gpurun_out/${TAG}_prof.err; exit 1; }
cd $R
timeout -k 10 200 python -u scripts/kt_timeline.py --record > gpurun_out/${TAG}_kt_timeline.txt 2>&1 || exit 1
fi
[ "$PART" = "A" ] && { echo done; exit 0; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_chol -o run -- python $R/scripts/chol_bench.py 5000 3 > $R/gpurun_out/${TAG}_chol.log 2>&1 || { echo "chol profile failed"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_phyprof -o run -- python3 $R/bench.py --workload phylo --steps 100 --warmup 100 --no-cpu > $R/gpurun_out/${TAG}_phyprof.json 2> $R/gpurun_out/${TAG}_phyprof.err || { echo "phylo rocprof failed"; tail -5 $R/gpurun_out/${TAG}_phyprof.err; exit 1; }
cd $R
timeout -k 10 300 python bench.py --workload phylo --steps 200 --warmup 200 > gpurun_out/${TAG}_config3.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --workload spatial --method GPP --steps 500 --warmup 50 > gpurun_out/${TAG}_config5_gpp.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --workload spatial --steps 20 --warmup 5 > gpurun_out/${TAG}_config5_full.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --workload spatial --method NNGP --steps 100 --warmup 20 > gpurun_out/${TAG}_config5_nngp.json 2>/dev/null || exit 1
cat gpurun_out/${TAG}_config3.json gpurun_out/${TAG}_config5_gpp.json gpurun_out/${TAG}_config5_full.json gpurun_out/${TAG}_config5_nngp.json
echo done
