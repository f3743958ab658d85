#!/bin/bash
# Round 3: the tree / adaptive chain engine -- parity against the fused kernels
# and the oracle, then bench lines of the chain-engine configs.  First failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 900 python -u -m pytest tests/test_chain.py tests/test_dispersion.py tests/test_adaptive.py \
    tests/test_secondary.py tests/test_path_trace.py -x -v -m gpu --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_chain.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_chain.log | tail -8; [ $rc -eq 0 ] || exit $rc
for c in G3 R3 P4 A3; do
    timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1
    rc=$?; tail -1 gpurun_out/bench_$c.log | cut -c1-330; [ $rc -eq 0 ] || exit $rc
done
