#!/bin/bash
# Build A/B variants of a ping-pong forward body (in parallel): each NAME=ARGS pair generates
# variants/fwdpp_NAME.h with `tools/gen_fwdpp.py ARGS` and links variants/lib_NAME.so with the two
# hd128 forward objects rebuilt against it; compare with tools/lib_ab.py (path@fwd_w4=2).
# With --fp8 first, the fp8 body (tools/gen_fwd8pp.py -> the fwd_fp8 object; path@fp8_w4=2).
#   tools/fwdpp_variants.sh "nosm=--abl nosm" "st=--stamps" ...
#   tools/fwdpp_variants.sh --fp8 "nosm=--abl nosm" ...
set -e
cd "$(dirname "$0")/.."
gen=tools/gen_fwdpp.py; def=XFA_FWDPP_BODY; objs="fwd:128:bf16 fwd:128:f16"
if [ "$1" = "--fp8" ]; then gen=tools/gen_fwd8pp.py; def=XFA_FWD8PP_BODY; objs=fwd_fp8; shift; fi
python xf_flash_attention_cutlass_amd/build.py --no-ext > /dev/null
mkdir -p variants
pids=()
for spec in "$@"; do
    name="${spec%%=*}"; args="${spec#*=}"
    python $gen $args --out "variants/fwdpp_$name.h" > /dev/null
    python tools/quick_variant.py "$name" "-D$def=\"$PWD/variants/fwdpp_$name.h\"" $objs > "variants/$name.log" 2>&1 &
    pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
ls -la variants/lib_*.so
