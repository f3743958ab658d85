#!/bin/bash
# GPU parity suite (one process, per-test time limit); optional -k filter in $1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
K=${1:+-k "$1"}
eval timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread $K > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -15; exit $rc
