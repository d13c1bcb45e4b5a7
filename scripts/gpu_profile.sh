#!/bin/bash
# One workload on one GPU: rocprofv3 kernel stats, the PMC passes (separate runs) and the bench line that reads them.
#   KEY=sedov_n400 ARGS="" scripts/gpu_profile.sh
#   KEY=evrard_n300 ARGS="--init evrard --side 300" scripts/gpu_profile.sh
# -> gpurun_out/prof_$KEY/ (kernel stats), gpurun_out/pmc_$KEY/summary.json (copy it to profiles/pmc_$KEY.json,
#    the file bench.py reads for this workload), gpurun_out/bench_$KEY.log (bench line with this build's counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
KEY=${KEY:?KEY=<init>_n<side>}
A=${ARGS:-}
mkdir -p gpurun_out
echo "== kernel stats $KEY"; date
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$KEY -o run -- python bench.py $A --steps 3 --warmup 1 --no-cpu-baseline --no-build-step > gpurun_out/prof_$KEY.log 2>&1 || { tail -5 gpurun_out/prof_$KEY.log; exit 1; }
if [ "${PMC:-1}" = "1" ]; then
  TAG=$KEY ARGS="$A --steps 2 --warmup 1 --no-cpu-baseline --no-build-step" bash scripts/gpu_pmc.sh || exit 1
  mkdir -p profiles && cp gpurun_out/pmc_$KEY/summary.json profiles/pmc_$KEY.json
fi
echo "== bench $KEY"; date
timeout -k 10 500 python bench.py $A ${BENCH_EXTRA:-} > gpurun_out/bench_$KEY.log 2>&1 || { tail -5 gpurun_out/bench_$KEY.log; exit 1; }
tail -1 gpurun_out/bench_$KEY.log
