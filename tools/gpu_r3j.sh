#!/bin/bash
# XCD-banded chain trace queue: chain-engine parity tests, then A/B on P4 / R3 / G3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests/test_chain.py tests/test_binning.py tests/test_path_trace.py tests/test_dispersion.py \
    tests/test_secondary.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_j.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_j.log; [ $rc -eq 0 ] || exit $rc
ab() {   # tag, config, rounds, switches...
    local tag=$1 cfg=$2 r=$3; shift 3
    AB_CONFIG=$cfg timeout -k 10 500 python tools/ab_bench.py "$@" --rounds $r > gpurun_out/abj_$tag.log 2>&1
    local rc=$?; echo "== $tag"; grep -v amdgpu.ids gpurun_out/abj_$tag.log | grep -E "^\{|^variant" | sed 's/counts.*primary SIMD/primary SIMD/' | cut -c1-240; return $rc
}
ab p4 P4 3 chain_bands=0,1 || exit $?
ab r3 R3 5 chain_bands=0,1 || exit $?
ab g3 G3 2 chain_bands=0,1 || exit $?
