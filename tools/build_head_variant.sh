#!/bin/bash
# Build the library of a git revision (default HEAD) into varlib/NAME.so for A/B runs
# (tools/ab_bench.sh).  usage: bash tools/build_head_variant.sh NAME [REV]
set -e
NAME=$1; REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/gsr_wt.XXXX)
git -C "$ROOT" worktree add -f -q "$WT" "$REV"
mkdir -p "$ROOT/varlib"
(cd "$WT" && python -c "from gsviewer_amd import build as b; b.build(out='$ROOT/varlib/$NAME.so')")
git -C "$ROOT" worktree remove --force "$WT"
