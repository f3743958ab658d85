#!/bin/bash
# PMC passes over the 1-GPU bench (one counter set per rocprofv3 pass, kernel
# trace only -- never combined with sys/runtime/hip/hsa tracing).  Each pass has
# its own time limit; a timeout / abort / fault ends the script, an unknown
# counter name only skips that pass.
# Outputs: gpurun_out/pmc/<pass>/..._counter_collection.csv, gpurun_out/pmc/counters.txt
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT" || exit 1
mkdir -p gpurun_out/pmc
export MRT_SCENE_CACHE=/tmp/mrt_scenes
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1
rc=$?; case $rc in 124|134|137|139) echo "rocprofv3 -L died rc=$rc"; exit $rc;; esac

pass() {
    local name="$1"; shift
    echo "== pass $name: $*"
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "gpurun_out/pmc/$name" -o run \
        -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "gpurun_out/pmc/$name.log" 2>&1
    local rc=$?
    tail -2 "gpurun_out/pmc/$name.log"
    case $rc in
        0) ;;
        124|134|137|139) echo "pass $name died rc=$rc -- stopping"; exit $rc;;
        *) echo "pass $name failed rc=$rc (skipped)";;
    esac
}

PASSES="${PMC_PASSES:-fetch write l2 sq l1 valu}"
want() { case " $PASSES " in *" $1 "*) return 0;; esac; return 1; }
want fetch && pass fetch FETCH_SIZE
want write && pass write WRITE_SIZE
want l2 && pass l2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
want sq && pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD
want l1 && pass l1 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM
want valu && pass valu SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE
want ta && pass ta TA_TA_BUSY_sum TA_BUSY_max TA_ADDR_STALLED_BY_TD_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE
want td && pass td TD_TD_BUSY_sum TD_TC_STALL_sum TD_LOAD_WAVEFRONT_sum TD_COALESCABLE_WAVEFRONT_sum GRBM_GUI_ACTIVE
want tcp && pass tcp TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE
want lvl && pass lvl SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH
exit 0
