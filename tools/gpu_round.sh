#!/bin/bash
# Bench legs for the new rows (R3 secondary rays, A3 adaptive supersampling),
# the default C3 bench, and rocprofv3 kernel-trace summaries of C3 and R3.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for c in R3 A3; do
    timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 > gpurun_out/bench_$c.log 2>&1
    rc=$?; tail -1 gpurun_out/bench_$c.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r3 -o run -- python3 bench.py --config R3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_r3.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_a3 -o run -- python3 bench.py --config A3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_a3.log 2>&1
exit $?
