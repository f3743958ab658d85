#!/bin/bash
# Batched dome sampling: full GPU suite, then libmrt.so (batched) vs libmrt_domeseq.so (sequential) on C5 / D1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
bash tools/gpu_pytest.sh || exit $?
echo "== C5"; AB_ROUNDS=2 AB_CONFIG=C5 bash tools/gpu_ab_libs.sh domeseq || exit $?
echo "== D1"; AB_ROUNDS=4 AB_CONFIG=D1 bash tools/gpu_ab_libs.sh domeseq || exit $?
