#!/bin/bash
# Round 4, first GPU call: the GPU parity suite, smoke, the C3 headline at the
# driver's settings, then kernel traces of C3 / C2 at the driver's settings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
bash tools/gpu_pytest.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_C3_driver.log 2>&1
rc=$?; tail -1 gpurun_out/bench_C3_driver.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
CONFIGS="${TRACE_CONFIGS:-C3 C2}" bash tools/gpu_steptrace.sh
