#!/bin/bash
# Round 4: parity suite (transparent shadows, material environment maps, round-3 walk
# back as the default), then the final scene at a reduced size with the chain levels'
# shadow rays inside chain_trace (0) and on the lane-refill kernel (1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
bash tools/gpu_pytest.sh || exit $?
for v in 0 1; do
  timeout -k 10 400 python bench.py --config FS --size 476x260 --steps 2 --warmup 1 --inflight 1 --latency-frames 1 \
    --no-cpu-baseline --tune chain_shadow_refill=$v > gpurun_out/bench_FS_small_csr$v.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_FS_small_csr$v.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_g3prof.sh
