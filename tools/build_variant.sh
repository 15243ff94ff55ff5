#!/bin/bash
# Build a libslk variant with extra -D flags into build_abl/<name>.so (profiling only), with the same
# per-source flags as the production build (splitcnn/build.py).
# usage: tools/build_variant.sh NAME "-DSLK_WIDE_XCD=0 ..."
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/build_abl"
python3 - "$ROOT" "$1" "$2" <<'PY'
import sys
root, name, flags = sys.argv[1], sys.argv[2], sys.argv[3]
sys.path.insert(0, root + "/split-learning-k8s_amd")
from splitcnn.build import build_library
print(build_library(out=f"{root}/build_abl/{name}.so", defines=flags.split()))
PY
