#!/bin/bash
# Host build throughput on the GPU box's CPU share (tools/build_bench.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
nproc; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
/tmp/spin 1 2>/dev/null
MRT_BUILD_TRACE=1 timeout -k 10 600 python3 tools/build_bench.py --out gpurun_out/build_bench.json
