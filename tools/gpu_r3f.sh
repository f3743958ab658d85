#!/bin/bash
# Binning key sweep (direction / origin bits) on P4 (chain levels) and C5 (frame shadow pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
ab() {   # config, rounds, switches...
    local cfg=$1 r=$2; shift 2
    AB_CONFIG=$cfg timeout -k 10 500 python tools/ab_bench.py "$@" --rounds $r > gpurun_out/abk_$cfg.log 2>&1
    local rc=$?; grep -v amdgpu.ids gpurun_out/abk_$cfg.log | grep -E "^\{" | cut -c1-240; return $rc
}
# bin_dbits+bin_obits pairs within 12 bits
K=2+0,2+1,2+2,3+0,3+1,3+2,4+0,4+1,5+0,6+0,0+4,1+3
ab P4 3 bin=0,6 bin_dbits+bin_obits=$K || exit $?
ab C5 2 bin=0,1 bin_dbits+bin_obits=$K || exit $?
