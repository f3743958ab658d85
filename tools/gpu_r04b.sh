#!/bin/bash
# Round 4: GPU parity suite, then an interleaved A/B of the merged-node build against
# the current one (each with the self-resetting tile counters off / on).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
bash tools/gpu_pytest.sh || exit $?
AB_ROUNDS=5 bash tools/gpu_ab_libs.sh merge self_reset=0,1 > gpurun_out/ab_merge_selfreset.txt 2>&1
rc=$?; cat gpurun_out/ab_merge_selfreset.txt | cut -c1-400; exit $rc
