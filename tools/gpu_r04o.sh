#!/bin/bash
# Round 4: object-space instance bin keys (bin_inst 2) -- binning equality tests, then
# an interleaved A/B on C5 (bin_inst 0 / 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests/test_binning.py -x -q -m gpu --timeout 240 --timeout-method thread \
  -k "identical_frames and (C5 or D1)" > gpurun_out/pytest_bin2.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_bin2.log; [ $rc -eq 0 ] || exit $rc
AB_CONFIG=C5 timeout -k 10 600 python tools/ab_bench.py bin_inst=0,2 --rounds 3 > gpurun_out/ab_bin2_C5.txt 2>&1
rc=$?; grep -E "^\{" gpurun_out/ab_bin2_C5.txt | cut -c1-220; [ $rc -eq 0 ] || exit $rc
AB_CONFIG=C5 timeout -k 10 600 python tools/ab_bench.py bin_inst=2,0 --rounds 3 > gpurun_out/ab_bin2_C5b.txt 2>&1
rc=$?; grep -E "^\{" gpurun_out/ab_bin2_C5b.txt | cut -c1-220; exit $rc
