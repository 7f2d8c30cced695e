#!/bin/bash
# PMC passes for the forward kernel variants; results under gpurun_out/pmc/<variant>_<pass>
# usage: bash tools/pmc_fwd.sh "fwd_pp=0" "fwd_pp=1" ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pmc
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS"
P3="TCC_EA0_RDREQ TCC_EA0_WRREQ TCC_HIT TCC_MISS"
for v in "$@"; do
  tag=$(echo "$v" | tr '=,' '__')
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P --output-format csv -d gpurun_out/pmc/${tag}_p$i -o run -- python3 tools/run_fwd.py --opt $v ${EXTRA} > gpurun_out/pmc/${tag}_p$i.log 2>&1 || { echo "FAILED $tag p$i"; exit 1; }
  done
done
echo done
