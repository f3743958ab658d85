#!/bin/bash
# GPU parity suite, then the R3 / A3 bench legs.  Each GPU step has its own
# time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in R3 A3; do
    timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 > gpurun_out/bench_$c.log 2>&1
    rc=$?; tail -1 gpurun_out/bench_$c.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
