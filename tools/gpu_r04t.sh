#!/bin/bash
# Round 4: (1) the per-launch counter clear as one fill (kCtrBytes padded to 256 B) against the
# unpadded length (libmrt_oddctr.so), C3 / C2 interleaved; (2) the C3 share model with
# bucket-batch launches sized for 1 / 2 / 4 tiles per wave (batch_tpw).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04t
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for cfg in C3 C2; do
  AB_CONFIG=$cfg AB_ROUNDS=3 bash tools/gpu_ab_libs.sh oddctr > gpurun_out/r04t/ab_oddctr_$cfg.txt 2>&1
  rc=$?; grep -E "^==|^\{" gpurun_out/r04t/ab_oddctr_$cfg.txt | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
for t in 1 2 4; do
  timeout -k 10 300 python -u bench.py --config C3 --share 2,4,8 --no-cpu-baseline --tune batch_tpw=$t > gpurun_out/r04t/share_tpw$t.json 2> gpurun_out/r04t/share_tpw$t.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04t/share_tpw$t.json')); print('tpw $t', {n: (v['predicted_speedup'], v['bound'], [p['ms_per_step'] for p in v['per_rank']]) for n, v in d['shares'].items()})"
done
