#!/bin/bash
# Round 4: frame kernel occupancy sweep on C2 and C3 (is C2's gain with 64 LDS nodes an
# occupancy effect?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for cfg in C2 C3; do
  echo "== $cfg"
  AB_CONFIG=$cfg timeout -k 10 300 python tools/ab_bench.py frame1_waves=5,6,7,8,7,5 --rounds 3 > gpurun_out/waves_$cfg.txt 2>&1
  rc=$?; grep -E "^\{" gpurun_out/waves_$cfg.txt | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
