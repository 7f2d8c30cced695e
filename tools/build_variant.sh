#!/bin/bash
# Build the library with a replacement kernel header and park it as a named variant for
# tools/lib_ab.py:  bash tools/build_variant.sh <name> <header-file> [target-header-name]
# (the tree is restored and rebuilt afterwards).
set -e
cd "$(dirname "$0")/.."
name=$1; hdr=$2; tgt=${3:-fmha_fwd_kernel.h}
C=xf_flash_attention_cutlass_amd/csrc
mkdir -p variants
cp $C/$tgt /tmp/_variant_keep.h
cp "$hdr" $C/$tgt
python -c "from xf_flash_attention_cutlass_amd import build; build.build_lib()" 
cp xf_flash_attention_cutlass_amd/lib/libpaged-attention.so variants/lib_$name.so
cp /tmp/_variant_keep.h $C/$tgt
touch $C/$tgt
python -c "from xf_flash_attention_cutlass_amd import build; build.build_lib()"
echo "variants/lib_$name.so"
