#!/bin/bash
# Build a libslk variant with extra -D flags into build_abl/<name>.so (profiling only).
# usage: tools/build_variant.sh NAME "-DSLK_WIDE_L=3 ..."
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/build_abl"
C="$ROOT/split-learning-k8s_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I "$ROOT/include" $2 \
  "$C/slk_client.hip" "$C/slk_server.hip" "$C/slk_optim.hip" "$C/slk_data.hip" "$C/slk_wide.hip" "$C/slk_wide_head.hip" "$C/slk_wino.hip" \
  -o "$ROOT/build_abl/$1.so"
echo "$ROOT/build_abl/$1.so"
