#!/bin/bash
# Build libmrt.so of git revision $1 into rendering-algorithms-raytracer_amd/lib/libmrt_$2.so
# (for two-library A/B runs with tools/gpu_ab_libs.sh).  Uses a scratch worktree.
set -e
REV=${1:?rev}; NAME=${2:?name}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/mrt_rev.XXXXXX)
git -C "$ROOT" worktree add -q --detach "$WT" "$REV"
make -C "$WT/rendering-algorithms-raytracer_amd" -s -j4 > /dev/null
cp "$WT/rendering-algorithms-raytracer_amd/lib/libmrt.so" "$ROOT/rendering-algorithms-raytracer_amd/lib/libmrt_$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built $REV -> lib/libmrt_$NAME.so"
