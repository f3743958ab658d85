#!/bin/bash
# One GPU session: parity tests, smoke, short bench, kernel-trace profile.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
echo "== pytest -m gpu" && \
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] && \
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -5 gpurun_out/smoke.log; [ $rc -eq 0 ] && \
echo "== bench" && timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?; tail -5 gpurun_out/bench.log; [ $rc -eq 0 ] && \
echo "== rocprof" && cd /tmp && export TMPDIR=/tmp && cd - > /dev/null && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?; tail -3 gpurun_out/prof.log; exit $rc
