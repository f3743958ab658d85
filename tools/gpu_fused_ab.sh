#!/bin/bash
# Round 3: parity of the fused one-launch C1-C3 path, then an interleaved A/B of
# frame1_kernel occupancy targets against the two-launch path (config C3), then
# one bench line at one and four frames in flight.  Each GPU step has its own
# time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py tests/test_abi_v4.py -x -q -m gpu \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fused.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_bench.py fused=0,1 frame1_waves=5,6,7,8 --rounds 5 > gpurun_out/ab_fused.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_fused.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline > gpurun_out/bench_if1.log 2>&1
rc=$?; tail -1 gpurun_out/bench_if1.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_if4.log 2>&1
rc=$?; tail -1 gpurun_out/bench_if4.log | cut -c1-600; exit $rc
