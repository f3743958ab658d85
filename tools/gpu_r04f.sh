#!/bin/bash
# Round 4: the final scene's kernel-time breakdown, the share model at 8 frames in
# flight, and C5 A/Bs (instance-major shadow-ray bins; 4-wave instanced primary kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 300 python -u -m pytest tests/test_binning.py tests/test_instancing.py -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_bin.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_bin.log; [ $rc -eq 0 ] || exit $rc
AB_CONFIG=C5 timeout -k 10 500 python tools/ab_bench.py bin_inst=0,1 primary_inst_waves=5,4 --rounds 3 > gpurun_out/ab_c5.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_c5.txt | grep "^{" | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config C3 --share 8 --steps 20 --warmup 5 --inflight 8 > gpurun_out/share_C3_if8.log 2>&1
rc=$?; tail -1 gpurun_out/share_C3_if8.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_fs_prof.sh
