#!/bin/bash
# GPU suite on the auto binning policy, then occupancy / frames-in-flight A/B on C3, C5, P4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
bash tools/gpu_pytest.sh || exit $?
ab() {   # tag, config, rounds, switches...
    local tag=$1 cfg=$2 r=$3; shift 3
    AB_CONFIG=$cfg timeout -k 10 500 python tools/ab_bench.py "$@" --rounds $r > gpurun_out/abg_$tag.log 2>&1
    local rc=$?; echo "== $tag"; grep -v amdgpu.ids gpurun_out/abg_$tag.log | grep -E "^\{" | cut -c1-240; return $rc
}
ab c3w C3 7 frame1_waves=5,6,7,8 || exit $?
ab c3i2 C3 5 frame1_waves=6 --inflight 2 || exit $?
ab c3i4 C3 5 frame1_waves=6 --inflight 4 || exit $?
ab c3i8 C3 5 frame1_waves=6 --inflight 8 || exit $?
ab c5 C5 2 primary_inst_waves=1,5,6 shadow_sched=-1,1 || exit $?
ab p4 P4 3 chain_trace_waves=1,8 || exit $?
