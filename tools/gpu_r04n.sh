#!/bin/bash
# Round 4: any-hit shadow walks of the frame kernel in near-first order (near_first=1)
# against the reference order (0), C3 / C3L / C2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for cfg in C3 C3L C2; do
  echo "== $cfg"
  AB_CONFIG=$cfg timeout -k 10 300 python tools/ab_bench.py near_first=0,1 --rounds 5 > gpurun_out/nf_$cfg.txt 2>&1
  rc=$?; grep -E "^\{|^variant" gpurun_out/nf_$cfg.txt | cut -c1-260; [ $rc -eq 0 ] || exit $rc
done
