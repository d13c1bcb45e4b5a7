#!/bin/bash
# A/B of in-tree library builds on one box, each twice in alternating order (same state, same clocks):
#   LIBS="lib lib_old" ARGS="" scripts/ab_libs.sh      -> per-kernel ms of each run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for L in ${LIBS:-lib}; do
    SPHEXA_AMD_LIB=$PWD/sph-exa_amd/$L/libsphexa_hip.so timeout -k 10 300 python bench.py ${ARGS:-} --steps ${STEPS:-4} --warmup ${WARMUP:-2} --no-cpu-baseline > gpurun_out/ab/$L.$rep.log 2> gpurun_out/ab/$L.$rep.err || { echo "$L failed"; tail -5 gpurun_out/ab/$L.$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['kernels_ms'].items() if v > 0.01}, 'sync', round(d['stages_ms']['sync'],2), 'ng', d['neighbors_per_particle'], 'kept', d['config'].get('neighbor_skin', {}).get('kept_frozen_clusters_per_step'), d['config'].get('neighbor_skin', {}).get('search_ms_per_step')); [print('   ', k, v) for k, v in d.get('kernels_ms_per_step', {}).items() if k != 'findNeighbors']" gpurun_out/ab/$L.$rep.log $L
    grep -h "search grid\|search-reps" gpurun_out/ab/$L.$rep.err | tail -2
  done
done
