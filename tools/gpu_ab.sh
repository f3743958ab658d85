#!/bin/bash
# GPU parity tests, then an interleaved A/B of tuning switches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] && \
timeout -k 10 400 python tools/ab_bench.py "$@" > gpurun_out/ab.log 2>&1; rc=$?; cat gpurun_out/ab.log | grep -v amdgpu.ids; exit $rc
