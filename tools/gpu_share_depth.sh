#!/bin/bash
# The C3 share model at several pipeline depths (--inflight buffers and streams per rank).
set -o pipefail
mkdir -p gpurun_out/share_depth
for d in 4 6 8 12; do
  echo "[share] inflight $d"
  timeout -k 10 300 python -u bench.py --config C3 --share 2,4,8 --inflight $d --no-cpu-baseline \
      > gpurun_out/share_depth/d$d.json 2> gpurun_out/share_depth/d$d.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/share_depth/d$d.json')); print('frame', d['frame']['ms_per_step'], {n: (v['predicted_speedup'], v['bound'], v['slowest_rank_ms'], v['mean_rank_ms']) for n, v in d['shares'].items()})"
done
