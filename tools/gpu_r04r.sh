#!/bin/bash
# Round 4: FS with its chain levels' dome shadow rays binned by default -- the final-scene and
# binning GPU tests, the remaining key variants at 476x260, then the full-size FS bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04r
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests/test_final_scene.py tests/test_binning.py -x -v -m gpu --timeout 300 \
  --timeout-method thread > gpurun_out/r04r/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04r/pytest.log; [ $rc -eq 0 ] || exit $rc
FS_REPS=3 timeout -k 10 400 python -u tools/fs_stats.py 476x260 bin=0 bin=4,bin_inst=1 bin=4,bin_inst=2 bin=4,bin_inst=0,chain_bands=1 \
  bin=4,chain_bands=0 > gpurun_out/r04r/fs_stats.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/r04r/fs_stats.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config FS --steps 1 --warmup 0 --inflight 1 --latency-frames 1 > gpurun_out/r04r/fs_bench.log 2> gpurun_out/r04r/fs_bench.err
rc=$?; tail -1 gpurun_out/r04r/fs_bench.log | cut -c1-200; exit $rc
