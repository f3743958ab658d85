#!/bin/bash
# R3 / A3 / P4 at 20 steps (noise check of the chain rewrite) + kernel trace of R3 and P4, one frame in flight.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for c in R3 A3 P4; do
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/b20_$c.log 2>&1
    rc=$?; tail -1 gpurun_out/b20_$c.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in R3 P4; do
    timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr_$c -o run \
        -- python3 bench.py --config $c --inflight 1 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/tr_$c.log 2>&1 || exit $?
done
