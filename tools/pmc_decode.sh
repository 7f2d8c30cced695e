#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pmcd
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
P2="TCC_HIT TCC_MISS TCC_EA0_RDREQ GRBM_GUI_ACTIVE"
P3="TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P --output-format csv -d gpurun_out/pmcd/p$i -o run -- python3 tools/decode_one.py > gpurun_out/pmcd/p$i.log 2>&1 || echo "FAILED p$i"
done
python3 tools/pmc_summary.py "gpurun_out/pmcd/p*" decode
