#!/bin/bash
# Full GPU suite on the cleaned-up kernels, then chain shading occupancy A/B (P4 / R3 / G3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
bash tools/gpu_pytest.sh || exit $?
ab() {   # tag, config, rounds, switches...
    local tag=$1 cfg=$2 r=$3; shift 3
    AB_CONFIG=$cfg timeout -k 10 500 python tools/ab_bench.py "$@" --rounds $r > gpurun_out/abm_$tag.log 2>&1
    local rc=$?; echo "== $tag"; grep -v amdgpu.ids gpurun_out/abm_$tag.log | grep -E "^\{" | cut -c1-240; return $rc
}
ab p4 P4 3 chain_shade_waves=1,2 bin_blocks=1,4 || exit $?
ab r3 R3 5 chain_shade_waves=1,2 || exit $?
ab g3 G3 2 chain_shade_waves=1,2 || exit $?
ab c5 C5 2 bin_blocks=1,2,4 || exit $?
echo "== instance entry fused with the next visit (libmrt.so) vs a step of its own (libmrt_oldentry.so), C5"
AB_ROUNDS=2 AB_CONFIG=C5 bash tools/gpu_ab_libs.sh oldentry || exit $?
