#!/bin/bash
# Build A/B variants of the 4-wave forward body (in parallel): each NAME=ARGS pair generates
# variants/fwd4_NAME.h with `tools/gen_fwd4.py ARGS` and links variants/lib_NAME.so with the two
# hd128 forward objects rebuilt against it (tools/quick_variant.py); compare with tools/lib_ab.py.
#   tools/fwd4_variants.sh "ks8=--ks 8 --vs 8 --lead 8 --npre 4 --nvpre 2" ...
set -e
cd "$(dirname "$0")/.."
python xf_flash_attention_cutlass_amd/build.py --no-ext > /dev/null
mkdir -p variants
pids=()
for spec in "$@"; do
    name="${spec%%=*}"; args="${spec#*=}"
    python tools/gen_fwd4.py $args --out "variants/fwd4_$name.h" > /dev/null
    python tools/quick_variant.py "$name" "-DXFA_FWD4_BODY=\"$PWD/variants/fwd4_$name.h\"" fwd:128:bf16 fwd:128:f16 > "variants/$name.log" 2>&1 &
    pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
ls -la variants/lib_*.so
