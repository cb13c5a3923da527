#!/bin/bash
# GPU-box helper: the z draw's compact LDS tables (z_kernel.h ZT_COMPACT) A/B in the table
# microbenchmark (time + LDS bank-conflict counters), then the product's z parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-zab}
mkdir -p $R/gpurun_out/${TAG}_zab
cd $R
for v in 0 1; do
  echo "== ZT_COMPACT=$v"
  timeout -k 10 120 scripts/ubench_ztab_c$v > gpurun_out/${TAG}_zab/c$v.txt 2>&1 || { cat gpurun_out/${TAG}_zab/c$v.txt; exit 1; }
  cat gpurun_out/${TAG}_zab/c$v.txt
done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES --kernel-include-regex "zt_kernel" --output-format csv \
    -d $R/gpurun_out/${TAG}_zab/pmc$v -o p -- $R/scripts/ubench_ztab_c$v > $R/gpurun_out/${TAG}_zab/pmc$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $R/gpurun_out/${TAG}_zab/pmc$v.log; exit 1; }
done
cd $R
python - <<PY
import csv, glob, collections
for v in (0, 1):
    f = glob.glob("gpurun_out/${TAG}_zab/pmc%d/**/*counter_collection.csv" % v, recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in sorted(acc.items()):
        m = {n: sum(x) / len(x) for n, x in c.items()}
        print("ZT_COMPACT=%d %-40s conflict %.3g / lds-active %.3g = %.1f%%  lds insts %.3g  valu %.3g" % (
            v, k[:40], m.get("SQ_LDS_BANK_CONFLICT", 0), m.get("SQ_LDS_IDX_ACTIVE", 1),
            100 * m.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, m.get("SQ_LDS_IDX_ACTIVE", 1)), m.get("SQ_INSTS_LDS", 0), m.get("SQ_INSTS_VALU", 0)))
PY
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_zpar.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_zpar.log; grep -E "FAILED" gpurun_out/${TAG}_zpar.log | head
case $rc in 0|1) ;; *) exit 1;; esac
