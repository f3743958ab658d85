#!/bin/bash
# Round 4: chain scratch budget A/B with estimated level capacities -- the default
# (48 GB cap per stream) against 8 GB per stream, on every chain-engine config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for cfg in R3 P4 G3; do
  for t in "" "--tune chain_mb=8192"; do
    timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline $t > gpurun_out/mb_ab.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/mb_ab.log; exit $rc; }
    tail -1 gpurun_out/mb_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', '${t:-default}', d['value'], d['ms_per_step'], d.get('frame_latency_ms'))"
  done
done
for t in "" "--tune chain_mb=8192"; do
  timeout -k 10 300 python bench.py --config FS --size 476x260 --steps 2 --warmup 1 --inflight 1 --latency-frames 1 \
    --no-cpu-baseline $t > gpurun_out/mb_ab.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/mb_ab.log; exit $rc; }
  tail -1 gpurun_out/mb_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('FS476', '${t:-default}', d['value'], d['ms_per_step'], d.get('frame_latency_ms'))"
done
