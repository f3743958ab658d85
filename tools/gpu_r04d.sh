#!/bin/bash
# Round 4: A/B of the scalar fetch of wave-uniform triangles (scalar_nodes 1 = nodes
# only, 3 = nodes + triangles) on C3 / C3L / C2, the share model of the split, and a
# short bench of the final scene (FS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_final_scene.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
for cfg in C3 C3L C2; do
  AB_CONFIG=$cfg timeout -k 10 300 python tools/ab_bench.py scalar_nodes=1,3 --rounds 5 > gpurun_out/ab_tri_$cfg.txt 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_tri_$cfg.txt | cut -c1-250; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --config C3 --share 2,4,8 --steps 20 --warmup 5 > gpurun_out/share_C3.log 2>&1
rc=$?; tail -1 gpurun_out/share_C3.log | cut -c1-3000; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config FS --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline > gpurun_out/bench_FS.log 2>&1
rc=$?; tail -1 gpurun_out/bench_FS.log | cut -c1-1500; exit $rc
