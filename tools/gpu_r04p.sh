#!/bin/bash
# Round 4: alpha test inlined into the walks (libmrt_ai.so) against the call (libmrt.so),
# on the final scene at 476x260 (alpha-mapped grass and leaves in every instance).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for i in 1 2; do
  for L in libmrt.so libmrt_ai.so; do
    MRT_LIB=rendering-algorithms-raytracer_amd/lib/$L timeout -k 10 300 python bench.py --config FS --size 476x260 --steps 2 \
      --warmup 1 --inflight 1 --latency-frames 1 --no-cpu-baseline > gpurun_out/ai.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/ai.log; exit $rc; }
    tail -1 gpurun_out/ai.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['value'], d['ms_per_step'], d['frame_latency_ms'])"
  done
done
