#!/bin/bash
# Modeled strong-split curves (bench.py --share) for the configs in $CONFIGS, one
# run per (config, frames per launch) in $FPL; lines to gpurun_out/share_<cfg>_k<K>.json.
# Each run has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
CONFIGS="${CONFIGS:-C3}"
FPL="${FPL:-1}"
WIDTHS="${WIDTHS:-2,4,8}"
for c in $CONFIGS; do
  for k in $FPL; do
    timeout -k 10 ${LIMIT:-400} python bench.py --config $c --share $WIDTHS --frames-per-launch $k \
        --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/share_${c}_k$k.log 2>&1
    rc=$?; tail -1 gpurun_out/share_${c}_k$k.log > gpurun_out/share_${c}_k$k.json
    python3 - "$c" "$k" <<'PY' || tail -3 gpurun_out/share_${c}_k$k.log
import json, sys
c, k = sys.argv[1:]
d = json.load(open(f"gpurun_out/share_{c}_k{k}.json"))
print(c, "K", k, "frame", d["frame"], {n: (s["step_ms_model"], s["bound"], s["predicted_speedup"]) for n, s in d["shares"].items()})
PY
    [ $rc -eq 0 ] || exit $rc
  done
done
