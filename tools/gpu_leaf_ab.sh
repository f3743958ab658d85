#!/bin/bash
# Flattened leaf loop of the instanced any-hit step: GPU suite, C5 / textures A/B of libmrt.so
# (flattened) vs libmrt_nested.so (per-slot packet loops), then the C3 profile at the new occupancy.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
bash tools/gpu_pytest.sh || exit $?
echo "== C5 leaf loop"; AB_ROUNDS=2 AB_CONFIG=C5 bash tools/gpu_ab_libs.sh nested > gpurun_out/ab_leaf_C5.log 2>&1 || exit $?
grep -E "^==|^\{" gpurun_out/ab_leaf_C5.log | cut -c1-200
rm -rf gpurun_out/prof3/C3
CONFIGS=C3 bash tools/prof_all.sh > gpurun_out/prof_c3.log 2>&1; rc=$?; grep -E "^== |failed" gpurun_out/prof_c3.log; exit $rc
