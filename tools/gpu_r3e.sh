#!/bin/bash
# Kernel-trace of the binned chain engine (R3, P4): the bin kernels' cost per level.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in R3 P4; do
    timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bt_$c -o run \
        -- python3 bench.py --config $c --inflight 1 --steps 4 --warmup 1 --no-cpu-baseline --tune bin=6 > gpurun_out/bt_$c.log 2>&1 || exit $?
done
for c in R3 P4; do
    echo "== $c"; python3 - "$c" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/bt_{sys.argv[1]}/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:9.2f} total_ms {float(r["TotalDurationNs"])/1e6:9.2f}')
PY
done
