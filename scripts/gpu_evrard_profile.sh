#!/bin/bash
# Evrard n=300 (BASELINE config 5, self-gravity) on one GPU: bench line, rocprofv3 kernel stats, PMC passes.
#   scripts/gpu_evrard_profile.sh -> gpurun_out/evr_bench.log, gpurun_out/evr_prof/, gpurun_out/pmc_evr/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
A="--init evrard --side 300 --no-cpu-baseline"
timeout -k 10 300 python bench.py $A --steps 5 --warmup 2 > gpurun_out/evr_bench.log 2>&1 || { tail -5 gpurun_out/evr_bench.log; exit 1; }
tail -1 gpurun_out/evr_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/evr_prof -o evr -- python bench.py $A --steps 3 --warmup 1 > gpurun_out/evr_prof.log 2>&1 || { tail -5 gpurun_out/evr_prof.log; exit 1; }
TAG=evr ARGS="$A --steps 2 --warmup 1" bash scripts/gpu_pmc.sh
