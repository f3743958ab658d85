#!/bin/bash
# Round 4: touching the next node's line before the leaf triangles (MRT_NODE_TOUCH 1 = vector
# load, 2 = scalar load for a wave-uniform next node) -- parity of those builds, then an
# interleaved A/B against the default build on C3 / C3L / C2 / C5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for v in touch1 touch2; do
MRT_LIB=rendering-algorithms-raytracer_amd/lib/libmrt_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  -x -q -m gpu --timeout 240 --timeout-method thread -k "not full" > gpurun_out/pytest_$v.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in touch1 touch2; do
for cfg in C3 C3L C2; do
  echo "== $v $cfg"
  AB_CONFIG=$cfg AB_ROUNDS=3 bash tools/gpu_ab_libs.sh $v > gpurun_out/ab_${v}_$cfg.txt 2>&1
  rc=$?; grep -E "^==|^\{" gpurun_out/ab_${v}_$cfg.txt | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
done
