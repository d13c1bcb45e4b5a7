#!/bin/bash
# A/B of library builds on the search: per-kernel times and (profile builds) the search's cycle breakdown.
#   LIBS="lib lib_old" ARGS="--side 200" scripts/ab_search.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for L in ${LIBS:-lib}; do
  for W in ${WARMS:-2 20}; do
    SPHEXA_AMD_LIB=sph-exa_amd/$L/libsphexa_hip.so timeout -k 10 200 python bench.py ${ARGS:---side 200} --steps ${STEPS:-4} --warmup $W --no-cpu-baseline > gpurun_out/ab/$L.$W.log 2> gpurun_out/ab/$L.$W.err || { echo "$L failed"; tail -5 gpurun_out/ab/$L.$W.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'warm', sys.argv[3], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['kernels_ms'].items() if v > 0.01}, 'cand', round(d['candidates_per_particle'],1), 'ng', d['neighbors_per_particle'])" gpurun_out/ab/$L.$W.log $L $W
    grep nsprof gpurun_out/ab/$L.$W.err | tail -1
  done
done
