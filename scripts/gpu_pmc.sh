#!/bin/bash
# PMC passes (separate runs, kernel-trace only; no sys/runtime trace -- see the HIP guide) over a short bench of the
# default workload, then the per-kernel summary bench.py reads (profiles/pmc_<key>.json after copying; scripts/gpu_profile.sh).
#   TAG=r2 scripts/gpu_pmc.sh      -> gpurun_out/pmc_$TAG/{p*/,summary.json,summary.txt}
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-x}
mkdir -p $OUT
ARGS=${ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-build-step}
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES"; do
  i=$((i+1))
  echo "== pass $i: $pmc"; date
  timeout -s KILL 240 rocprofv3 --pmc $pmc --output-format csv -d $OUT/p$i -o pmc -- python bench.py $ARGS > $OUT/p$i.log 2>&1 || { rc=$?; tail -5 $OUT/p$i.log; exit $rc; }
done
python scripts/pmc_summary.py $OUT $OUT/summary.json > $OUT/summary.txt && cat $OUT/summary.txt
echo done
