#!/bin/bash
# Round 3: ray binning + dome replay -- the full GPU suite, then interleaved A/B
# of the switches per config.  First failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
bash tools/gpu_pytest.sh || exit $?
ab() {   # config, rounds, switches...
    local cfg=$1 r=$2; shift 2
    AB_CONFIG=$cfg timeout -k 10 400 python tools/ab_bench.py "$@" --rounds $r > gpurun_out/ab_$cfg.log 2>&1
    local rc=$?; grep -v amdgpu.ids gpurun_out/ab_$cfg.log | grep -E "^\{|^variant" | cut -c1-260; return $rc
}
ab C5 3 dome_replay=0,1 bin=0,1 || exit $?
ab D1 5 dome_replay=0,1 bin=0,1 || exit $?
ab C4 5 bin=0,1 || exit $?
ab P4 3 bin=0,2,4,6 || exit $?
ab R3 5 bin=0,6 || exit $?
ab G3 3 bin=0,6 || exit $?
