#!/bin/bash
# G3: chain scratch budget per stream (fewer chunks of units per adaptive pass), then fresh
# bench lines of A3 R3 P4 G3 (their tracked rocprof fields).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
AB_CONFIG=G3 timeout -k 10 500 python tools/ab_bench.py chain_mb=16384,32768,49152 --rounds 2 > gpurun_out/ab_g3mb.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_g3mb.log | grep -E "^\{" | cut -c1-240; [ $rc -eq 0 ] || exit $rc
CONFIGS="A3 R3 P4 G3" EXTRA="--steps 10 --warmup 2" bash tools/gpu_bench_all.sh
