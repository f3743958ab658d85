#!/bin/bash
# The N > 1 bench path rehearsed on one GPU (bench.py MRT_BENCH_REHEARSE=gloo): every rank on
# cuda:0, collectives over gloo through host copies.  Runs the split (one frame per step) at
# N = 2 through bench.py's own launcher and at N = 4 through torch.distributed.run, and the
# weak-scaling batch split at N = 2.  Lines land in gpurun_out/rehearse/.
set -e -o pipefail
mkdir -p gpurun_out/rehearse
export MRT_BENCH_REHEARSE=gloo
echo "[rehearse] N=2 split frame (bench.py launcher)"
timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/rehearse/n2_frame.json 2> gpurun_out/rehearse/n2_frame.err
tail -c 600 gpurun_out/rehearse/n2_frame.json
echo "[rehearse] N=4 split frame (torch.distributed.run)"
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 4 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/rehearse/n4_frame.json 2> gpurun_out/rehearse/n4_frame.err
tail -c 600 gpurun_out/rehearse/n4_frame.json
echo "[rehearse] N=2 split batch, G3"
timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --split batch --config G3 \
    > gpurun_out/rehearse/n2_batch_g3.json 2> gpurun_out/rehearse/n2_batch_g3.err
tail -c 600 gpurun_out/rehearse/n2_batch_g3.json
echo "[rehearse] done"
