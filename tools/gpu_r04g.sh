#!/bin/bash
# Round 4: parity suite (uniform-stack walk, chain shadow refill), the final scene at a
# reduced size, then an interleaved A/B of the round-3 walk (libmrt_v1.so) against the
# new one on C3 / C3L / C2 / C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
bash tools/gpu_pytest.sh || exit $?
timeout -k 10 600 python bench.py --config FS --size 476x260 --steps 2 --warmup 1 --inflight 1 --latency-frames 1 --no-cpu-baseline > gpurun_out/bench_FS_small.log 2>&1
rc=$?; tail -1 gpurun_out/bench_FS_small.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
for cfg in C3 C3L C2 C4; do
  echo "== $cfg"
  AB_CONFIG=$cfg AB_ROUNDS=3 bash tools/gpu_ab_libs.sh v1 > gpurun_out/ab_walk_$cfg.txt 2>&1
  rc=$?; grep -E "^==|^\{" gpurun_out/ab_walk_$cfg.txt | cut -c1-220; [ $rc -eq 0 ] || exit $rc
done
