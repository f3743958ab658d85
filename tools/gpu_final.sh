#!/bin/bash
# Round-end evidence on the round's last binary (run after tools/prof_all.sh, whose
# summaries bench.py reads for the tracked fields).  PART=1: GPU parity suite, smoke,
# then the C3 headline at the driver's own settings and C2 / C3L at the same 20-step
# region; PART=2: one bench line per remaining config (10 steps) and FS (one frame).
# Every line carries the CPU baseline.  Each GPU step has its own time limit; the first
# failure ends the script.  Lines go to gpurun_out/bench_<cfg>.log (last line = JSON).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MRT_SCENE_CACHE=/tmp/mrt_scenes
line() {   # config, time limit, bench arguments...
    local c=$1 lim=$2; shift 2
    timeout -k 10 $lim python bench.py --config $c "$@" > gpurun_out/bench_$c.log 2>&1
    local rc=$?
    tail -1 gpurun_out/bench_$c.log | cut -c1-160
    [ $rc -eq 0 ] || { echo "$c bench failed rc=$rc -- stopping"; exit $rc; }
}
if [ "${PART:-1}" = 1 ]; then
    bash tools/gpu_pytest.sh || exit $?
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    rc=$?; tail -1 gpurun_out/smoke.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
    # the driver's command: no --config (C3), 20 steps after 5 warmups
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_C3.log 2>&1
    rc=$?; tail -1 gpurun_out/bench_C3.log | cut -c1-160; [ $rc -eq 0 ] || exit $rc
    line C2 300 --steps 20 --warmup 5
    line C3L 300 --steps 20 --warmup 5
else
    for c in ${CONFIGS:-C4 D1 C5 A3 R3 P4 G3}; do line $c 400 --steps 10 --warmup 2; done
    [ -n "${NO_FS:-}" ] || line FS 600 --steps 1 --warmup 0 --inflight 1
fi
exit 0
