#!/bin/bash
# Round-4 GPU session: focused tests (TESTS), optional Evrard bench line (EVRARD=1), optional A/B (LIBS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  echo "== tests: $TESTS"; date
  timeout -k 10 ${FOCUS_T:-700} python -u -m pytest $TESTS -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/focus.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|ranks vs|Error" $OUT/focus.log | tail -60
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ "${EVRARD:-0}" = "1" ]; then
  echo "== evrard bench"; date
  timeout -k 10 300 python bench.py --init evrard --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_evrard.json 2> $OUT/bench_evrard.err || { rc=$?; tail -5 $OUT/bench_evrard.err; exit $rc; }
fi
if [ -n "${LIBS:-}" ]; then
  echo "== A/B: $LIBS"; date
  LIBS="$LIBS" bash scripts/ab_libs.sh || exit $?
fi
echo "== done"; date
