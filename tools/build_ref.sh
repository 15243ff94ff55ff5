#!/bin/bash
# Build libslk.so from the sources of git revision REF (profiling A/B: old vs new in one process) into
# ab/NAME.so, with the production flags (splitcnn/build.py of that revision).
# usage: tools/build_ref.sh REF NAME
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REF=$1; NAME=$2
WT=/tmp/slk_wt_$NAME
rm -rf "$WT"; git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add --detach "$WT" "$REF" > /dev/null
mkdir -p "$ROOT/ab"
python3 - "$WT" "$ROOT/ab/$NAME.so" <<'PY'
import sys
wt, out = sys.argv[1], sys.argv[2]
sys.path.insert(0, wt + "/split-learning-k8s_amd")
from splitcnn.build import build_library
print(build_library(out=out))
PY
git -C "$ROOT" worktree remove --force "$WT"
