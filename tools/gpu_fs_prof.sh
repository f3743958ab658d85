#!/bin/bash
# Kernel-time breakdown of the final scene (FS) at a reduced size (rocprofv3
# kernel trace + stats only).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/fsprof
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -s KILL 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fsprof/trace -o run \
    -- python3 bench.py --config FS --size ${FS_SIZE:-476x260} --steps 1 --warmup 0 --inflight 1 --latency-frames 1 --no-cpu-baseline \
    > gpurun_out/fsprof/bench.log 2>&1
rc=$?; tail -1 gpurun_out/fsprof/bench.log | cut -c1-300
f=$(find gpurun_out/fsprof/trace -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:25]: print('%-90s %8s calls %10.2f ms total %9.1f us avg' % (r['Name'][:90], r['Calls'], float(r['TotalDurationNs'])/1e6, float(r['AverageNs'])/1e3))
"
exit $rc
