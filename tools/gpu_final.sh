#!/bin/bash
# Round-end evidence: GPU parity suite, smoke, and single-stream rocprofv3
# kernel-trace summaries of the A3 / R3 legs (one frame in flight, so each
# kernel's average duration is its own launch time).  Each GPU step has its
# own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in A3 R3; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1_$c -o run -- python3 bench.py --config $c --steps 5 --warmup 2 --inflight 1 --no-cpu-baseline > gpurun_out/prof1_$c.log 2>&1
    rc=$?; tail -1 gpurun_out/prof1_$c.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
