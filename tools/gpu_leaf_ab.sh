#!/bin/bash
# Flattened leaf loop of the instanced any-hit step: C5 A/B of libmrt.so (flattened) vs
# libmrt_nested.so (per-slot packet loops); then the C3 profile at the new occupancy and
# fresh C3 (driver settings) / C5 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
echo "== C5 leaf loop"; AB_ROUNDS=2 AB_CONFIG=C5 bash tools/gpu_ab_libs.sh nested > gpurun_out/ab_leaf_C5.log 2>&1 || exit $?
grep -E "^==|^\{" gpurun_out/ab_leaf_C5.log | cut -c1-200
rm -rf gpurun_out/prof3/C3
CONFIGS=C3 bash tools/prof_all.sh > gpurun_out/prof_c3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_C3_driver.log 2>&1 || exit $?
tail -1 gpurun_out/bench_C3_driver.log | cut -c1-200
CONFIGS="C5" EXTRA="--steps 10 --warmup 2" bash tools/gpu_bench_all.sh
