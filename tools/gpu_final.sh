#!/bin/bash
# Round-end evidence, part 1: GPU parity suite, smoke, then one bench line per
# config with the CPU baseline (the C3 headline at the driver's own settings).
# Part 2 is tools/prof_all.sh (rocprofv3 kernel trace + PMC passes per config).
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
bash tools/gpu_pytest.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_C3_driver.log 2>&1
rc=$?; tail -1 gpurun_out/bench_C3_driver.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
CONFIGS="${CONFIGS:-C2 C4 D1 C5 A3 R3 P4 G3}" EXTRA="--steps 10 --warmup 2" bash tools/gpu_bench_all.sh
