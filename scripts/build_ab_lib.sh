#!/bin/bash
# Build libf110.so of an earlier commit for in-process A/B runs (scripts/lib_ab.py, gpu_run.sh's
# libab / abhead steps): a temporary git worktree of COMMIT, the _build.py flags and sources,
# output OUT (default ab_libs/head.so; *.so files are git-ignored but travel with gpurun).
#
#   bash scripts/build_ab_lib.sh HEAD~3 ab_libs/head.so
set -euo pipefail
COMMIT=${1:?commit}
OUT=${2:-ab_libs/head.so}
REPO=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/f110_ab_XXXXXX)
trap 'git -C "$REPO" worktree remove --force "$WT" >/dev/null 2>&1 || true' EXIT
git -C "$REPO" worktree add --detach "$WT" "$COMMIT" >/dev/null
mkdir -p "$(dirname "$REPO/$OUT")"
cd "$WT"
python3 - "$REPO/$OUT" <<'PY'
import os, subprocess, sys
sys.path.insert(0, os.getcwd())
from f110_gymnasium_ros2_jazzy_amd import _build as B
cmd = [B.hipcc()] + B.FLAGS + [os.path.join(B.CSRC, f) for f in B.SOURCES] + ["-o", sys.argv[1]]
subprocess.run(cmd, check=True)
print("built", sys.argv[1])
PY
