#!/bin/bash
# Bench variants on one box (same process image, back-to-back): BENCH_ARGS is a
# ';'-separated list of bench.py argument sets.  First failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
IFS=';' read -ra SETS <<< "${BENCH_ARGS:---steps 20}"
i=0
for a in "${SETS[@]}"; do
    echo "== bench $a"
    timeout -k 10 300 python bench.py --no-cpu-baseline $a > gpurun_out/ab_$i.log 2>&1
    rc=$?; grep '^{' gpurun_out/ab_$i.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(json.dumps({k:d[k] for k in ('value','ms_per_step')}), json.dumps(d['launch_ms']), json.dumps(d.get('wave_timing_us')))"
    [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_$i.log; exit $rc; }
    i=$((i+1))
done
exit 0
