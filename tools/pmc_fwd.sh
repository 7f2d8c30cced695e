#!/bin/bash
# PMC passes for forward/backward kernel configurations; results under
# gpurun_out/pmc/<tag>_p<pass> (summarise with tools/pmc_summary.py).
# usage: bash tools/pmc_fwd.sh <tag> [run_fwd.py args...]
#   e.g. bash tools/pmc_fwd.sh c2 ; bash tools/pmc_fwd.sh nc --noncausal ; bash tools/pmc_fwd.sh bwd --mode bwd
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pmc
tag=$1; shift
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d gpurun_out/pmc/${tag}_p$i -o run -- python3 tools/run_fwd.py "$@" > gpurun_out/pmc/${tag}_p$i.log 2>&1 || { echo "FAILED $tag p$i"; exit 1; }
done
echo "pmc $tag done"
