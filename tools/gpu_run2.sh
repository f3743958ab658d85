set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/diag_runtime.py torch-first > gpurun_out/diag1.log 2>&1; echo "diag1 rc=$?"; cat gpurun_out/diag1.log | grep -v amdgpu.ids
timeout -k 10 120 python tools/diag_runtime.py mrt-first > gpurun_out/diag2.log 2>&1; echo "diag2 rc=$?"; cat gpurun_out/diag2.log | grep -v amdgpu.ids
bash tools/gpu_check.sh
