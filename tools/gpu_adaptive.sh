#!/bin/bash
# GPU parity suite, then the A3 (adaptive supersampling) and C3 bench legs.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config A3 --steps 5 --warmup 2 > gpurun_out/bench_a3.log 2>&1
rc=$?; tail -2 gpurun_out/bench_a3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log; exit $rc
