#!/bin/bash
# Kernel traces of the driver's own bench settings (20 timed steps after 5 warmup
# steps, frames in flight as bench.py runs them), one rocprofv3 run per config in
# $CONFIGS, summarised by tools/step_trace.py into gpurun_out/steptrace.json
# (busy union per timed step, overlap, per-step roofline fractions).
# Kernel trace only (never combined with sys / runtime / hip / hsa tracing or PMC);
# each run has its own time limit; a failure ends the script.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT" || exit 1
OUT=${OUT:-gpurun_out/steptrace}
mkdir -p $OUT
export MRT_SCENE_CACHE=/tmp/mrt_scenes
CONFIGS="${CONFIGS:-C3 C2 C4 D1 C5 A3 R3 P4 G3}"
for cfg in $CONFIGS; do
    rm -rf "$OUT/$cfg"
    mkdir -p "$OUT/$cfg"
    # the config's frames in flight as hardware queues (bench.py sets them itself, but under rocprofv3 the
    # HIP runtime starts before bench.py runs, so the variable has to be in the environment already)
    q=$(python3 -c "import sys; sys.path.insert(0, 'rendering-algorithms-raytracer_amd'); from miro import scenes; print(max(4, scenes.CONFIGS['$cfg'].get('inflight', 4)))")
    GPU_MAX_HW_QUEUES=$q timeout -s KILL ${LIMIT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$cfg/trace" -o run \
        -- python3 bench.py --gpus 1 --config "$cfg" --steps 20 --warmup 5 --no-cpu-baseline $BENCH_EXTRA \
        > "$OUT/$cfg/bench.log" 2>&1
    rc=$?
    tail -1 "$OUT/$cfg/bench.log" | cut -c1-160
    [ $rc -eq 0 ] || { echo "$cfg trace failed rc=$rc -- stopping"; exit $rc; }
    python3 tools/step_trace.py "$OUT/$cfg/trace" "$OUT/$cfg/bench.log" "$cfg" "$OUT/steptrace.json" > "$OUT/$cfg/summary.json" \
        || { echo "$cfg summary failed"; exit 1; }
    python3 -c "import json; r=json.load(open('$OUT/$cfg/summary.json')); print('$cfg', 'union/step', r['busy_union_ms_per_step'], 'ms', 'step', r['ms_per_step_traced_run'], 'union/step', r['union_over_step'], 'overlap', r['kernel_sum_over_union'], 'frac_l2', r.get('frac_l2_per_step'))"
done
exit 0
