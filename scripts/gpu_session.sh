#!/bin/bash
# One GPU-box session: GPU parity tests, smoke, the default bench line and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout ends the script (test *failures* do not).
#   TAG=r2a scripts/gpu_session.sh     outputs under gpurun_out/$TAG/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-session}
mkdir -p $OUT
if [ "${TESTS:-1}" = "1" ]; then
  echo "== pytest -m gpu"; date
  timeout -k 10 ${PYTEST_T:-900} python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  echo "== smoke"; date
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { rc=$?; cat $OUT/smoke.log; exit $rc; }
  cat $OUT/smoke.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  echo "== bench"; date
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 || { rc=$?; tail -20 $OUT/bench.log; exit $rc; }
  tail -1 $OUT/bench.log
fi
if [ "${PROF:-1}" = "1" ]; then
  echo "== rocprofv3 kernel trace"; date
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof.log 2>&1 || { rc=$?; tail -20 $OUT/prof.log; exit $rc; }
  find $OUT/prof -name "*kernel_stats.csv"
fi
echo "== done"; date
