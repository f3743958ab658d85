#!/bin/bash
# Per-config rocprofv3 evidence for bench.py's roofline (summarised by
# tools/prof3.py into profiles/<round>_<cfg>_rocprof.txt + profiles/<round>_profile.json).
# For each config in $CONFIGS, every run is `bench.py --config CFG --inflight 1`
# (one frame in flight, so a dispatch's duration is its own launch time):
#   trace  --kernel-trace --stats        (durations, VGPR / SGPR / LDS / scratch columns)
#   fetch  --pmc FETCH_SIZE              write  --pmc WRITE_SIZE   (separate passes: TCC slots)
#   sq     --pmc <SQ wave-state + TCP + GRBM counters>             (latency evidence)
# Counters are checked against `rocprofv3 -L` first; absent ones are dropped.
# Kernel trace only: never combined with sys / runtime / hip / hsa tracing.  Each
# run has its own time limit; a timeout / abort / fault ends the script.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT" || exit 1
OUT=${OUT:-gpurun_out/prof3}
mkdir -p $OUT
export MRT_SCENE_CACHE=/tmp/mrt_scenes
CONFIGS="${CONFIGS:-C3 C2 C4 D1 C5 A3 R3 P4 G3}"
STEPS="${STEPS:-6}"

timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1
have() { grep -qw -- "$1" $OUT/counters.txt || grep -qw -- "${1%_sum}" $OUT/counters.txt; }
SQ=""
for c in SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
         SQ_INSTS_VMEM_RD TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE; do
    if have $c; then SQ="$SQ $c"; else echo "counter $c not listed -- dropped"; fi
done
echo "sq pass counters:$SQ"

run() {
    local cfg="$1" name="$2" lim="$3"; shift 3
    echo "== $cfg $name: $*"
    timeout -s KILL $lim rocprofv3 "$@" --output-format csv -d "$OUT/$cfg/$name" -o run \
        -- python3 bench.py --config "$cfg" --inflight 1 --steps "$STEPS" --warmup 1 --no-cpu-baseline $BENCH_EXTRA \
        > "$OUT/$cfg/$name.log" 2>&1
    local rc=$?
    tail -1 "$OUT/$cfg/$name.log" | cut -c1-200
    case $rc in
        0) ;;
        *) echo "$cfg $name failed rc=$rc -- stopping"; exit $rc;;
    esac
}

for cfg in $CONFIGS; do
    mkdir -p "$OUT/$cfg"
    run "$cfg" trace 300 --kernel-trace --stats
    cp "$OUT/$cfg/trace.log" "$OUT/$cfg/bench.log"
    run "$cfg" fetch 300 --kernel-trace --pmc FETCH_SIZE
    run "$cfg" write 300 --kernel-trace --pmc WRITE_SIZE
    [ -n "$SQ" ] && run "$cfg" sq 300 --kernel-trace --pmc $SQ
done
exit 0
