#!/bin/bash
# Round-2 baseline on a fresh box: GPU parity suite + C3 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in C3 C4; do
timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1
rc=$?; tail -1 gpurun_out/bench_$c.log; [ $rc -eq 0 ] || exit $rc
done
