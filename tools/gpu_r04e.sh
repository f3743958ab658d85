#!/bin/bash
# Round 4: share model of the split (self-resetting counters off / on) and a
# reduced-size run of the final scene (FS) to size its full bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for t in 0 1; do
  timeout -k 10 300 python bench.py --config C3 --share 2,4,8 --steps 20 --warmup 5 --tune self_reset=$t > gpurun_out/share_C3_sr$t.log 2>&1
  rc=$?; tail -1 gpurun_out/share_C3_sr$t.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('self_reset $t frame', d['frame'])
for n,v in d['shares'].items(): print(n, v['slowest_rank_ms'], v['step_ms_model'], v['predicted_speedup'], [(r['ms_per_step'], r['host_issue_ms_per_step'], r['launch_alone_ms']) for r in v['per_rank'][:2]])"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python bench.py --config FS --size 476x260 --steps 2 --warmup 1 --inflight 1 --latency-frames 1 --no-cpu-baseline > gpurun_out/bench_FS_small.log 2>&1
rc=$?; tail -1 gpurun_out/bench_FS_small.log | cut -c1-1200; exit $rc
