#!/bin/bash
# round 6: the IPC split rehearsed through bench.py's own N = 2 launcher on one GPU (gloo,
# every rank on cuda:0), then the modeled 8-GPU curves (--share) with direct writes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MRT_SCENE_CACHE=/tmp/mrt_scenes
mkdir -p gpurun_out/share
MRT_BENCH_REHEARSE=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/share/rehearse_n2.log 2>&1
rc=$?; tail -1 gpurun_out/share/rehearse_n2.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for spec in ${SPECS:-C3:1 C3:8 C4:1 C5:1}; do
  c=${spec%%:*}; k=${spec#*:}
  st=20; [ $c = C3 ] || st=10
  timeout -k 10 600 python bench.py --config $c --share 2,4,8 --frames-per-launch $k --steps $st --warmup 3 \
      --no-cpu-baseline > gpurun_out/share/${c}_k$k.log 2>&1
  rc=$?; tail -1 gpurun_out/share/${c}_k$k.log > gpurun_out/share/${c}_k$k.json
  python - gpurun_out/share/${c}_k$k.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print(d["config"]["config"], "K", d["config"]["frames_per_launch"], "frame", d["frame"]["ms_per_step"],
      {n: (v["predicted_speedup"], v["bound"], v["slowest_rank_ms"]) for n, v in d["shares"].items()})
PY
  [ $rc -eq 0 ] || exit $rc
done
