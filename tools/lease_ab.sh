#!/bin/bash
# One lease: the default bench line, then the forward schedule A/B (in-process, interleaved) for
# bf16 C2 and the fp8 C2 shape: static XCD-paired persistent (default), per-XCD dynamic queues
# (fwd_dyn=2), and one workgroup per item (fwd_persistent=0, the reference's plain grid).
# usage: bash tools/lease_ab.sh <tag>      -> gpurun_out/<tag>_{bench,ab}.log
set -o pipefail
tag=${1:-lease}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -5 gpurun_out/${tag}_bench.log; exit 1; }
tail -1 gpurun_out/${tag}_bench.log | cut -c1-200
for m in fwd fwd_fp8; do
  timeout -k 10 200 python tools/perf_ab.py --mode $m --rounds 9 --iters 20 --prewarm 2 \
    --var "" --var fwd_dyn=2 --var fwd_persistent=0 >> gpurun_out/${tag}_ab.log 2>&1 || { tail -5 gpurun_out/${tag}_ab.log; exit 1; }
done
timeout -k 10 200 python tools/perf_ab.py --mode fwd --noncausal --rounds 5 --iters 10 --prewarm 1 \
  --var "" --var fwd_dyn=2 --var fwd_persistent=0 >> gpurun_out/${tag}_ab.log 2>&1 || { tail -5 gpurun_out/${tag}_ab.log; exit 1; }
cat gpurun_out/${tag}_ab.log
