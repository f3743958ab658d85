set -o pipefail
export MRT_SCENE_CACHE=/tmp/mrt_scenes
for c in C3 C3L; do for i in 1 2; do for L in libmrt libmrt_r04 libmrt_oct; do
  echo "== $c $L run $i"; AB_CONFIG=$c MRT_LIB=rendering-algorithms-raytracer_amd/lib/$L.so timeout -k 10 200 python tools/ab_bench.py --rounds 5 2>&1 | grep -E "^\{" || exit 1
done; done; done
