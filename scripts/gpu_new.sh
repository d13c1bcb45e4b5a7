#!/bin/bash
# Focused GPU run: the listed test files verbosely (-s: the trajectory metrics), then the whole -m gpu suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
echo "== focused: ${TESTS}"; date
timeout -k 10 ${FOCUS_T:-600} python -u -m pytest ${TESTS} -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/focus.log 2>&1
rc=$?; echo "focused rc=$rc"; grep -E "PASSED|FAILED|ERROR|L1|time rel|Sedov" $OUT/focus.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${SUITE:-1}" = "1" ]; then
  echo "== full suite"; date
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -8 $OUT/pytest_gpu.log
fi
echo "== done"; date
