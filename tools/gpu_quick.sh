#!/bin/bash
# GPU parity tests + default bench + frame-batch benches (world 1, batch path).
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; tail -2 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
for f in ${BATCH_FRAMES:-2 8}; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --frames $f > gpurun_out/bench_f$f.log 2>&1
    rc=$?; tail -1 gpurun_out/bench_f$f.log; [ $rc -eq 0 ] || exit $rc
done
exit 0
