#!/bin/bash
# C5's L2 behaviour per kernel on the round's final binary: one rocprofv3 --pmc pass (TCC hit /
# miss / EA read requests; kernel trace only), summarised by tools/pmc_summary.py-style parsing
# below into gpurun_out/c5_tcc.txt.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
cd "$ROOT" || exit 1
export MRT_SCENE_CACHE=/tmp/mrt_scenes
mkdir -p gpurun_out/c5tcc
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv \
    -d gpurun_out/c5tcc/pmc -o run -- python3 bench.py --config C5 --inflight 1 --steps 3 --warmup 1 --no-cpu-baseline \
    --latency-frames 1 > gpurun_out/c5tcc/bench.log 2>&1 || exit $?
python3 - <<'PY'
import csv, collections, re
rows = list(csv.DictReader(open("gpurun_out/c5tcc/pmc/run_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    agg[r["Kernel_Name"]][(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
out = ["# C5, rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum, bench.py --config C5 "
       "--inflight 1 --steps 3 --warmup 1 (round 6 final binary). Mean per dispatch."]
for k, d in agg.items():
    per = collections.defaultdict(list)
    for (c, _), v in d.items():
        per[c].append(v)
    m = {c: sum(v) / len(v) for c, v in per.items()}
    h, mi = m.get("TCC_HIT_sum", 0), m.get("TCC_MISS_sum", 0)
    name = re.sub(r"\(.*", "", k)[:70]
    out.append("%-72s L2 hit %.3f  hits %.3g  misses %.3g  EA read requests %.3g" % (name, h / max(1, h + mi), h, mi,
                                                                                  m.get("TCC_EA0_RDREQ_sum", 0)))
open("gpurun_out/c5_tcc.txt", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
