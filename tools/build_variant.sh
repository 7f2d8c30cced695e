#!/bin/bash
# Build the library with extra compile flags and park it as a named variant for
# tools/lib_ab.py:  bash tools/build_variant.sh <name> "<flags>"   e.g. "-DXFA_EXP_SCALAR=2"
# (objects are rebuilt with the flags, then the default build is restored).
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2
mkdir -p variants
XFA_EXTRA_FLAGS="$flags" python -c "from xf_flash_attention_cutlass_amd import build; build.build_lib(force=True)"
cp xf_flash_attention_cutlass_amd/lib/libpaged-attention.so variants/lib_$name.so
python -c "from xf_flash_attention_cutlass_amd import build; build.build_lib(force=True)"
echo "variants/lib_$name.so"
