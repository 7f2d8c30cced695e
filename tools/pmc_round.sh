#!/bin/bash
# Round profile of bench.py, per mode: a rocprofv3 kernel-trace --stats run, two SQ/GRBM PMC
# passes (instruction mix, waits, LDS, MFMA busy) and two TCC passes (FETCH_SIZE, WRITE_SIZE
# do not fit one pass on gfx950).  Each pass is its own run (rocprofv3 does not split passes).
# Output under gpurun_out/prof/<mode>_{stats,sq1,sq2,fetch,write}; summarise with
# tools/pmc_report.py.   usage: bash tools/pmc_round.sh fwd fwd_nc fwdbwd varlen decode
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof
SQ1="SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
SQ2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
for m in "$@"; do
  case $m in decode_ragged) MA="--mode decode --ragged";; fwd_nc) MA="--mode fwd --no-causal";; fwd_paged) MA="--mode fwd --page 16";; fwd_alibi) MA="--mode fwd --alibi";; fwd_window) MA="--mode fwd --window-left 1023";; *) MA="--mode $m";; esac
  B="bench.py $MA --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-monitor --prewarm-s 0.5"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${m}_stats -o run -- python3 $B > gpurun_out/prof/${m}_stats.out 2>&1 || { echo "FAILED stats $m"; exit 1; }
  echo "stats $m"
  for P in sq1 sq2 fetch write; do
    case $P in sq1) C="$SQ1";; sq2) C="$SQ2";; fetch) C="FETCH_SIZE";; write) C="WRITE_SIZE";; esac
    timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/prof/${m}_$P -o run -- python3 $B > gpurun_out/prof/${m}_$P.out 2>&1 || { echo "FAILED $P $m"; exit 1; }
    echo "$P $m"
  done
done
