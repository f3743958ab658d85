#!/bin/bash
# Round 4: chain chunks on estimated level capacities (+ fused fallback): the chain /
# transparency / dispersion tests first, then the whole suite, then G3 at the default
# and an 8 GB chunk budget with and without the estimates.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 600 python -u -m pytest tests/test_chain.py tests/test_transparent.py -x -q -m gpu --timeout 240 \
  --timeout-method thread > gpurun_out/pytest_chain.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_chain.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_pytest.sh || exit $?
for t in "" "--tune chain_mb=8192" "--tune chain_mb=8192 --tune chain_est=0"; do
  timeout -k 10 300 python bench.py --config G3 --no-cpu-baseline $t > gpurun_out/g3_est.log 2>&1
  rc=$?; echo "G3 $t"; tail -1 gpurun_out/g3_est.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('frame_latency_ms'), d.get('chain', ''))"; [ $rc -eq 0 ] || exit $rc
done
