#!/bin/bash
# Round profile: for each bench mode, a rocprofv3 kernel-trace --stats run of bench.py and
# two PMC passes (FETCH_SIZE, WRITE_SIZE — they do not fit one TCC pass on gfx950).
# Output under gpurun_out/prof/<mode>_{stats,fetch,write}; summarise with tools/traffic.py.
# usage: bash tools/profile_round.sh fwd decode ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof
for m in "$@"; do
  B="bench.py --mode $m --steps 10 --warmup 3 --no-cpu-baseline --no-extras"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${m}_stats -o run -- python3 $B > gpurun_out/prof/${m}_stats.log 2>&1 || { echo "FAILED stats $m"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/${m}_fetch -o run -- python3 $B > gpurun_out/prof/${m}_fetch.log 2>&1 || { echo "FAILED fetch $m"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/${m}_write -o run -- python3 $B > gpurun_out/prof/${m}_write.log 2>&1 || { echo "FAILED write $m"; exit 1; }
  echo "profiled $m"
done
