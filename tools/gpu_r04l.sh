#!/bin/bash
# Round 4: the stackless walk (libmrt_lds.so, MRT_LDS_NODES=16) -- parity of that build
# (hits, pixels, node / leaf visit counts against the oracle), then an interleaved A/B
# against the stack walk on C3 / C3L / C2 / C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
MRT_LIB=rendering-algorithms-raytracer_amd/lib/libmrt_lds.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  -x -q -m gpu --timeout 240 --timeout-method thread -k "not full" > gpurun_out/pytest_lds.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_lds.log; [ $rc -eq 0 ] || exit $rc
for v in lds lds64; do
for cfg in C3 C3L C2; do
  echo "== $v $cfg"
  AB_CONFIG=$cfg AB_ROUNDS=3 bash tools/gpu_ab_libs.sh $v > gpurun_out/ab_${v}_$cfg.txt 2>&1
  rc=$?; grep -E "^==|^\{" gpurun_out/ab_${v}_$cfg.txt | cut -c1-220; [ $rc -eq 0 ] || exit $rc
done
done
