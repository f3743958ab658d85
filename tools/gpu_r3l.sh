#!/bin/bash
# Leaf steps of the lane-refill shadow kernel: parity, then A/B on C5 / D1 (refill) and C4 (refill vs bands).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests/test_binning.py tests/test_gpu_parity.py tests/test_textures.py tests/test_instancing.py \
    -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_l.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_l.log; [ $rc -eq 0 ] || exit $rc
ab() {   # tag, config, rounds, switches...
    local tag=$1 cfg=$2 r=$3; shift 3
    AB_CONFIG=$cfg timeout -k 10 500 python tools/ab_bench.py "$@" --rounds $r > gpurun_out/abl_$tag.log 2>&1
    local rc=$?; echo "== $tag"; grep -v amdgpu.ids gpurun_out/abl_$tag.log | grep -E "^\{|^variant" | sed 's/counts.*primary SIMD/primary SIMD/' | cut -c1-240; return $rc
}
ab c5 C5 3 leaf_steps=0,1 || exit $?
ab d1 D1 5 leaf_steps=0,1 || exit $?
ab c4 C4 5 shadow_sched+leaf_steps=1+0,2+0,2+1 || exit $?
