#!/bin/bash
# Build a ping-pong probe variant: tools/gen_pingpong.py ARGS -> body_NAME.h -> libpp_NAME.so
#   bash tools/probe/build.sh NAME [gen_pingpong.py args]
set -e
cd "$(dirname "$0")"
name=${1:-base}; shift || true
python ../gen_pingpong.py --out body_$name.h "$@" > /dev/null
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared pingpong.hip -o libpp_$name.so \
  -DPP_BODY="\"body_$name.h\"" -Rpass-analysis=kernel-resource-usage 2> resource_$name.txt
echo "libpp_$name.so: $(grep -E 'remark: .*(VGPRs:|Spill:)' resource_$name.txt | sed 's/.*remark: //;s/ \[.*//' | sort -u | tr '\n' ' ')"
