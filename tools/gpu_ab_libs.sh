#!/bin/bash
# Alternate A/B runs of two library builds on one box (same device).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
A=rendering-algorithms-raytracer_amd/lib/libmrt.so
B=rendering-algorithms-raytracer_amd/lib/libmrt_$1.so
shift
for i in 1 2; do
  for L in $A $B; do
    echo "== $L run $i" && MRT_LIB=$L timeout -k 10 200 python tools/ab_bench.py "$@" --rounds ${AB_ROUNDS:-5} 2>&1 | grep -v amdgpu.ids | grep -E "^\{" || exit 1
  done
done
