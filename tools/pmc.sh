#!/bin/bash
# Per-config evidence for bench.py's roofline: for each config in $CONFIGS
# (default: all bench configs) one rocprofv3 --kernel-trace --stats run and two
# PMC passes (FETCH_SIZE, WRITE_SIZE -- separate runs; TCC budget), kernel trace
# only, never combined with sys/runtime/hip/hsa tracing.  Each run has its own
# time limit; a timeout / abort / fault ends the script.
# Outputs: gpurun_out/pmc/<cfg>/{trace,fetch,write}/..., summarised by tools/pmc_summary.py
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT" || exit 1
mkdir -p gpurun_out/pmc
export MRT_SCENE_CACHE=/tmp/mrt_scenes
CONFIGS="${CONFIGS:-C3 C2 C4 D1 C5 A3 R3 P4 G3}"
STEPS="${STEPS:-5}"

run() {
    local cfg="$1" name="$2"; shift 2
    echo "== $cfg $name: $*"
    timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "gpurun_out/pmc/$cfg/$name" -o run \
        -- python3 bench.py --config "$cfg" --steps "$STEPS" --warmup 1 --no-cpu-baseline \
        > "gpurun_out/pmc/$cfg/$name.log" 2>&1
    local rc=$?
    tail -1 "gpurun_out/pmc/$cfg/$name.log" | cut -c1-160
    case $rc in
        0) ;;
        124|134|137|139) echo "$cfg $name died rc=$rc -- stopping"; exit $rc;;
        *) echo "$cfg $name failed rc=$rc -- stopping"; exit $rc;;
    esac
}

for cfg in $CONFIGS; do
    mkdir -p "gpurun_out/pmc/$cfg"
    run "$cfg" trace --kernel-trace --stats
    run "$cfg" fetch --kernel-trace --pmc FETCH_SIZE
    run "$cfg" write --kernel-trace --pmc WRITE_SIZE
done
exit 0
