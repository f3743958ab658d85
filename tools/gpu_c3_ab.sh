#!/bin/bash
# C3 headline: interleaved A/B of the frame kernel's scalar node fetch and occupancy target.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
AB_CONFIG=C3 timeout -k 10 500 python tools/ab_bench.py scalar_nodes=0,1 frame1_waves=6,7 --rounds 9 > gpurun_out/ab_c3.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_c3.log | grep -E "^\{" | cut -c1-240; exit $rc
