#!/bin/bash
# C3 headline: frames in flight (HIP streams) sweep through bench.py itself, twice, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for rep in 1 2; do
  for n in 1 2 3 4 5 6 8 12 16; do
    timeout -k 10 120 python bench.py --config C3 --steps 200 --warmup 10 --inflight $n --no-cpu-baseline > gpurun_out/inf_$n.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/inf_$n.log').read().strip().splitlines()[-1]); print('inflight', $n, 'rep', $rep, d['value'], 'Mray/s', d['ms_per_step'], 'ms/step')"
  done
done
