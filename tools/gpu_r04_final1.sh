#!/bin/bash
# Round 4 final evidence, part 1: the GPU suite and smoke() on the final binary, one
# bench line per config (C3 at the driver's command), the C3 share model, and the final
# scene at 1904x1042.  Every step has its own limit; a failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final
mkdir -p $OUT
export MRT_SCENE_CACHE=/tmp/mrt_scenes
bash tools/gpu_pytest.sh || exit $?
cp gpurun_out/pytest_gpu.log $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
run() {   # cfg, limit, args...
  local cfg=$1 lim=$2; shift 2
  timeout -k 10 $lim python -u bench.py --config $cfg "$@" > $OUT/bench_$cfg.log 2> $OUT/bench_$cfg.err
  local rc=$?
  tail -1 $OUT/bench_$cfg.log > $OUT/$cfg.json
  python3 -c "import json; d=json.load(open('$OUT/$cfg.json')); r=d.get('roofline',{}); print('$cfg', d['value'], d['unit'], d['ms_per_step'], 'ms', 'lat', d.get('frame_latency_ms'), 'frac', r.get('frac'), 'per_step', (r.get('per_step') or {}).get('frac_l2'))" || true
  [ $rc -eq 0 ] || { echo "$cfg rc=$rc"; tail -5 $OUT/bench_$cfg.err; exit $rc; }
}
run C3 300 --gpus 1 --steps 20 --warmup 5
for cfg in C2 C3L C4 D1 C5 A3 R3 P4 G3; do run $cfg 400 --steps 10 --warmup 2; done
timeout -k 10 400 python -u bench.py --config C3 --share 2,4,8 --no-cpu-baseline > $OUT/share_C3.json 2> $OUT/share_C3.err
rc=$?; python3 -c "import json; d=json.load(open('$OUT/share_C3.json')); print({n: (v['predicted_speedup'], v['bound'], v['slowest_rank']) for n, v in d['shares'].items()})"; [ $rc -eq 0 ] || exit $rc
run FS 900 --steps 1 --warmup 0 --inflight 1 --latency-frames 1
