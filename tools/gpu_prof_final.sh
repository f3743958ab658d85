#!/bin/bash
# Round-end evidence, part 2: rocprofv3 kernel trace + PMC passes of $CONFIGS (tools/prof_all.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/prof_all.sh > gpurun_out/prof_${TAG:-x}.log 2>&1
rc=$?; grep -E "^== |failed" gpurun_out/prof_${TAG:-x}.log | tail -40; exit $rc
