#!/bin/bash
# Round 3 step: shim C5 + parity tests, tile-order A/B (serial + 4 in flight), and
# the C3 rocprofv3 evidence run (tools/prof_all.sh).  First failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests/test_shim.py tests/test_gpu_parity.py tests/test_abi_v4.py -x -q -m gpu \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_r3b.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r3b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_bench.py tile_lpt=0,1 --rounds 7 > gpurun_out/ab_lpt.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_lpt.log | tail -2; [ $rc -eq 0 ] || exit $rc
CONFIGS=C3 bash tools/prof_all.sh > gpurun_out/prof_c3.log 2>&1
rc=$?; tail -8 gpurun_out/prof_c3.log; exit $rc
