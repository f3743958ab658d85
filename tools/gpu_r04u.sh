#!/bin/bash
# Round 4: motion blur under a dome light (CHECK for motion-blurred lanes), the stepped instanced
# shadow walk in the chain trace (chain_shadow_step): equality on FS, then FS timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04u
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests/test_motion_blur.py tests/test_final_scene.py -x -v -m gpu --timeout 300 \
  --timeout-method thread > gpurun_out/r04u/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r04u/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
FS_REPS=3 timeout -k 10 500 python -u tools/fs_stats.py 476x260 chain_shadow_step=1 chain_shadow_step=0 chain_shadow_step=1 \
  > gpurun_out/r04u/fs_stats.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/r04u/fs_stats.log | cut -c1-150; exit $rc
