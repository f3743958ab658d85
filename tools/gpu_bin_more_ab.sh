#!/bin/bash
# Frame shadow-pass binning at key (2, 2) on C4 (rect light, 16 samples) and D1 (dome, no
# instances), and C5's primary occupancy (spill writes vs time).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
ab() {   # tag, config, rounds, switches...
    local tag=$1 cfg=$2 r=$3; shift 3
    AB_CONFIG=$cfg timeout -k 10 500 python tools/ab_bench.py "$@" --rounds $r > gpurun_out/abz_$tag.log 2>&1
    local rc=$?; echo "== $tag"; grep -v amdgpu.ids gpurun_out/abz_$tag.log | grep -E "^\{" | cut -c1-240; return $rc
}
ab c4 C4 5 bin=0,1 || exit $?
ab d1 D1 5 bin=0,1 || exit $?
ab c5 C5 2 primary_inst_waves=1,5 || exit $?
