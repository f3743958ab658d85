#!/bin/bash
# Same-box A/B of library builds: the libraries named in $LIBS (default: this build,
# libmrt.so, against round 4's libmrt_r04.so built from commit 981f1bb; libmrt_prev.so =
# a build of the last commit, from a git worktree) on each config of $CONFIGS,
# alternated twice; then tuning A/Bs given as "CFG:key=v1,v2" words in $TUNES.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for c in ${CONFIGS:-C3}; do for i in 1 2; do for L in ${LIBS:-libmrt libmrt_r04}; do
  echo "== $c $L run $i"
  AB_CONFIG=$c MRT_LIB=rendering-algorithms-raytracer_amd/lib/$L.so timeout -k 10 240 python tools/ab_bench.py \
      --rounds ${ROUNDS:-4} 2>&1 | grep -E "^(\{|variant)" || exit 1
done; done; done
for t in $TUNES; do
  c=${t%%:*}; kv=${t#*:}
  echo "== $c $kv"
  AB_CONFIG=$c timeout -k 10 300 python tools/ab_bench.py $kv --rounds ${ROUNDS:-4} 2>&1 | grep -E "^(\{|variant)" || exit 1
done
