#!/bin/bash
# GPU parity suite (one process, per-test time limit); optional -k expression in $1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
args=(tests -x -v -rP -m gpu --timeout 240 --timeout-method thread)
[ -n "$1" ] && args+=(-k "$1")
timeout -k 10 1200 python -u -m pytest "${args[@]}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -25; exit $rc
