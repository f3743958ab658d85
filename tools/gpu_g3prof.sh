#!/bin/bash
# G3 chain-engine breakdown: kernel statistics of one frame in flight at the default
# chunk budget and at an 8 GB budget (rocprofv3 kernel trace only), plus the bench
# lines of both at the driver's settings.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT" || exit 1
OUT=gpurun_out/g3prof
mkdir -p $OUT
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for mb in 0 8192; do
  extra=""; [ $mb -gt 0 ] && extra="--tune chain_mb=$mb"
  timeout -k 10 300 python3 bench.py --config G3 --no-cpu-baseline $extra > $OUT/bench_$mb.log 2>&1
  rc=$?; tail -1 $OUT/bench_$mb.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
  rm -rf $OUT/t$mb
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t$mb -o run \
      -- python3 bench.py --config G3 --steps 3 --warmup 1 --inflight 1 --latency-frames 1 --no-cpu-baseline $extra \
      > $OUT/prof_$mb.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "prof $mb rc=$rc"; exit $rc; }
  f=$(find $OUT/t$mb -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{r["Name"][:80]:80s} {int(r["Calls"]):6d} calls {float(r["TotalDurationNs"])/1e6:10.2f} ms {float(r["AverageNs"])/1e3:10.1f} us')
PY
done
