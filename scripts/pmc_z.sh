#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) for the dominant kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}
REGEX=${2:-z_wave|eta_fused|beta_lambda_wave|side_chain|g_eta_reduce|slab_pack}
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES"; do
  i=$((i+1))
  # (counter passes serialise the dispatches: the side chain's device-side joins inside a
  # sweep graph would wait on launches queued behind it, so the passes keep the graph edges;
  # the library then also copies the record by host-issued copies, not by waiting kernels)
  HMSC_SIDE_EDGES=1 HMSC_KERNEL_COPY=0 timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "$REGEX" --output-format csv \
    -d $R/gpurun_out/$TAG/p$i -o p -- python $R/scripts/trace_sweeps.py > $R/gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $R/gpurun_out/$TAG/p$i.log; exit 1; }
done
echo pmc done
