#!/bin/bash
# Full GPU parity suite + default bench line (HEAD health check).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log; exit $rc
