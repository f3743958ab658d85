#!/bin/bash
# Kernel trace of one config (default R3) at one frame in flight: per-kernel totals and the last frame's dispatches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
C=${1:-R3}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ctrace_$C -o run -- python3 bench.py --config $C --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline > gpurun_out/ctrace_$C.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/ctrace_$C -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py $f ${2:-60} > gpurun_out/ctrace_$C.txt
cat gpurun_out/ctrace_$C.txt
