#!/bin/bash
# Round 3: the cost-ordered tile queue of frame1_kernel (tile_lpt) against the
# plain queue (interleaved A/B, config C3), plus the fused-path parity tests and
# the bench line at one / four frames in flight.  Each GPU step has its own time
# limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "every_kernel or configs or full_hd or c1" \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_lpt.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_lpt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_bench.py tile_lpt=0,1 frame1_waves=5,6 --rounds 7 > gpurun_out/ab_lpt.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_lpt.log | tail -4; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline > gpurun_out/bench_if1.log 2>&1
rc=$?; tail -1 gpurun_out/bench_if1.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_if4.log 2>&1
rc=$?; tail -1 gpurun_out/bench_if4.log | cut -c1-300; exit $rc
