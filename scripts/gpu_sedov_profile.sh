#!/bin/bash
# Sedov -n 400 (the metric's workload) on one GPU at HEAD: rocprofv3 kernel stats, the five PMC passes, then the
# default bench line (which reads the PMC summary once it is copied to profiles/pmc_latest.json).
#   scripts/gpu_sedov_profile.sh -> gpurun_out/sed_prof/, gpurun_out/pmc_sed/, gpurun_out/sed_bench.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sed_prof -o sed -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sed_prof.log 2>&1 || { tail -5 gpurun_out/sed_prof.log; exit 1; }
TAG=sed ARGS="--steps 2 --warmup 1 --no-cpu-baseline" bash scripts/gpu_pmc.sh || exit 1
cp gpurun_out/pmc_sed/summary.json profiles/pmc_latest.json
timeout -k 10 400 python bench.py > gpurun_out/sed_bench.log 2>&1 || { tail -5 gpurun_out/sed_bench.log; exit 1; }
tail -1 gpurun_out/sed_bench.log
