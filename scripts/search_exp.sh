#!/bin/bash
# Search-cost experiments: the search repeated SX_SEARCH_REPS times (no h iteration) with parts switched off
# (NsArgs::experiment bits: 1 no list append, 2 no union rewrite, 4 no distance test, 8 no candidate stream,
# 16 no tree walk), for each library build in LIBS.
#   LIBS="lib lib_x" EXPS="0 1 2 4 8" ARGS="--side 400" scripts/search_exp.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sexp
for L in ${LIBS:-lib}; do
  for e in ${EXPS:-0 1 2 3 4 8}; do
    SPHEXA_AMD_LIB=sph-exa_amd/$L/libsphexa_hip.so SX_SEARCH_REPS=${REPS:-5} SX_SEARCH_EXP=$e timeout -k 10 300 python bench.py ${ARGS:---side 400} --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/sexp/$L.e$e.log 2> gpurun_out/sexp/$L.e$e.err || { echo "$L exp $e failed"; tail -5 gpurun_out/sexp/$L.e$e.err; exit 1; }
    echo "$L $(grep search-reps gpurun_out/sexp/$L.e$e.err | tail -1)"
  done
done
