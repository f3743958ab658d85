#!/bin/bash
# round 6 final: bench.py's N-rank launchers rehearsed on one GPU (gloo), the modeled N-GPU
# curves of the IPC split, and FS's chain-trace lane use under the shadow-walk schedules.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MRT_SCENE_CACHE=/tmp/mrt_scenes
mkdir -p gpurun_out/share
SPECS="C3:8 C3:1 C4:8 C5:8" bash tools/gpu_share_ipc.sh || exit $?
MRT_BENCH_REHEARSE=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 6 --warmup 2 --no-cpu-baseline \
    > gpurun_out/share/rehearse_n4.log 2>&1
rc=$?; grep '^{' gpurun_out/share/rehearse_n4.log | tail -1 | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/fs_stats.py chain_shadow_refill=1 chain_shadow_refill=0,chain_shadow_step=1 > gpurun_out/share/fs_stats.txt 2>&1
rc=$?; cat gpurun_out/share/fs_stats.txt | grep variant; exit $rc
