#!/bin/bash
# Build A/B variants of the ping-pong forward body (in parallel): each NAME=ARGS pair generates
# variants/fwdpp_NAME.h with `tools/gen_fwdpp.py ARGS` and links variants/lib_NAME.so with the two
# hd128 forward objects rebuilt against it; compare with tools/lib_ab.py (path@fwd_w4=2).
#   tools/fwdpp_variants.sh "nomix=--no-dmamix" ...
set -e
cd "$(dirname "$0")/.."
python xf_flash_attention_cutlass_amd/build.py --no-ext > /dev/null
mkdir -p variants
pids=()
for spec in "$@"; do
    name="${spec%%=*}"; args="${spec#*=}"
    python tools/gen_fwdpp.py $args --out "variants/fwdpp_$name.h" > /dev/null
    python tools/quick_variant.py "$name" "-DXFA_FWDPP_BODY=\"$PWD/variants/fwdpp_$name.h\"" fwd:128:bf16 fwd:128:f16 > "variants/$name.log" 2>&1 &
    pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
ls -la variants/lib_*.so
