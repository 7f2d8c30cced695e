#!/bin/bash
# Build a 16x16x32 ping-pong probe variant: tools/gen_pingpong16.py ARGS -> body16_NAME.h -> libpp16_NAME.so
#   bash tools/probe/build16.sh NAME [gen_pingpong16.py args]
set -e
cd "$(dirname "$0")"
name=${1:-base}; shift || true
python ../gen_pingpong16.py --out body16_$name.h "$@" > /dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared pingpong16.hip -o libpp16_$name.so \
  -DPP_BODY="\"body16_$name.h\"" -Rpass-analysis=kernel-resource-usage 2> resource16_$name.txt
echo "libpp16_$name.so: $(grep -E 'remark: .*(VGPRs:|Spill:)' resource16_$name.txt | sed 's/.*remark: //;s/ \[.*//' | sort -u | tr '\n' ' ')"
