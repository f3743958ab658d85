#!/bin/bash
# A/B of the wavefront shadow-kernel schedules (frames checked identical).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for c in ${CONFIGS:-C4 D1 C5}; do
    AB_CONFIG=$c timeout -k 10 400 python tools/ab_bench.py ${VARIANTS:-shadow_sched=0,1,2} --rounds ${ROUNDS:-3} > gpurun_out/ab_$c.log 2>&1
    rc=$?; echo "== $c"; grep -v "^variant" gpurun_out/ab_$c.log | tail -6; grep "^variant" gpurun_out/ab_$c.log | sed 's/counts.*primary SIMD/primary SIMD/'; [ $rc -eq 0 ] || exit $rc
done
