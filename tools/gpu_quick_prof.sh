#!/bin/bash
# Bench lines for $CONFIGS and one rocprofv3 kernel-trace --stats of each (kernel split).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
CONFIGS="${CONFIGS:-C3 D1 C5 R3}"
[ -n "$NOBENCH" ] || CONFIGS="$CONFIGS" EXTRA="--steps 10 --warmup 2 --no-cpu-baseline" bash tools/gpu_bench_all.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in $CONFIGS; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/qprof_$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --inflight 1 --no-cpu-baseline > gpurun_out/qprof_$c.log 2>&1
    rc=$?; [ $rc -eq 0 ] || exit $rc
    f=$(find gpurun_out/qprof_$c -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:8]:
    print('$c', r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')"
done
