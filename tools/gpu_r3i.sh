#!/bin/bash
# C3: fixed vs per-step cost of the timed region (steps sweep at the driver's warmup), and host cost per launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for n in 4 8; do
  for k in 5 10 20 40 100; do
    timeout -k 10 120 python bench.py --config C3 --steps $k --warmup 5 --inflight $n --no-cpu-baseline > gpurun_out/st_$n_$k.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/st_$n_$k.log').read().strip().splitlines()[-1]); print('inflight', $n, 'steps', $k, d['value'], 'Mray/s', d['ms_per_step'], 'ms/step')"
  done
done
timeout -k 10 120 python tools/diag_launch.py > gpurun_out/diag_launch.log 2>&1; rc=$?; cat gpurun_out/diag_launch.log | grep -v amdgpu.ids; exit $rc
