#!/bin/bash
# Round 4: GPU parity suite (C3L, full-size C5, device-side share assembly, final
# scene), then bench lines of C3 / C3L / C5 and the single-GPU share model of the
# 8-GPU split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
bash tools/gpu_pytest.sh || exit $?
CONFIGS="C3 C3L C5" EXTRA="--steps 20 --warmup 5 --no-cpu-baseline" bash tools/gpu_bench_all.sh || exit $?
timeout -k 10 300 python bench.py --config C3 --share 2,4,8 --steps 20 --warmup 5 > gpurun_out/share_C3.log 2>&1
rc=$?; tail -1 gpurun_out/share_C3.log | cut -c1-1500; exit $rc
