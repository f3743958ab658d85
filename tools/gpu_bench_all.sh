#!/bin/bash
# One bench line per config ($CONFIGS), each under its own time limit; the first
# failure ends the script.  Lines go to gpurun_out/bench_<cfg>.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
CONFIGS="${CONFIGS:-C3 C2 C4 D1 C5 A3 R3 P4 G3}"
EXTRA="${EXTRA:---steps 5 --warmup 1 --no-cpu-baseline}"
for c in $CONFIGS; do
    timeout -k 10 400 python bench.py --config $c $EXTRA > gpurun_out/bench_$c.log 2>&1
    rc=$?; tail -1 gpurun_out/bench_$c.log > gpurun_out/bench_$c.json
    python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_$c.json')); r=d['roofline']; print('$c', d['value'], 'Mray/s', d['ms_per_step'], 'ms/step', 'lat', d.get('frame_latency_ms'), 'l2', r['frac'], 'lane', r['lane_util'], d['launch_ms'])" 2>/dev/null || tail -3 gpurun_out/bench_$c.log
    [ $rc -eq 0 ] || exit $rc
done
