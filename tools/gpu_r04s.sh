#!/bin/bash
# Round 4: dispersive scenes bin their chain levels' shadow rays by default -- the binning,
# dispersion and chain GPU tests, then the G3 and FS bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04s
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests/test_binning.py tests/test_dispersion.py tests/test_chain.py tests/test_final_scene.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > gpurun_out/r04s/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r04s/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config G3 --steps 10 --warmup 2 > gpurun_out/r04s/g3.log 2> gpurun_out/r04s/g3.err
rc=$?; tail -1 gpurun_out/r04s/g3.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
AB_CONFIG=C4 timeout -k 10 300 python -u tools/ab_bench.py bin=-1,1 --rounds 3 > gpurun_out/r04s/c4_bin_ab.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/r04s/c4_bin_ab.log | grep "^{" | cut -c1-220; exit $rc
