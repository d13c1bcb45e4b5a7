#!/bin/bash
# Quick GPU check of a change: selected GPU tests (TESTS=...), then a short bench of the default workload.
#   TESTS="tests/test_gpu_parity.py tests/test_gpu_search_builds.py" scripts/gpu_quick.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  echo "== pytest $TESTS"; date
  timeout -k 10 ${PYTEST_T:-600} python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/quick_tests.log
  if [ $rc -ne 0 ]; then grep -E "^E |Error|FAILED" gpurun_out/quick_tests.log | head -30; exit $rc; fi
fi
if [ -n "${PRE:-}" ]; then echo "== $PRE"; timeout -k 10 500 $PRE || exit 1; fi
if [ "${BENCH:-1}" = "1" ]; then
  echo "== bench"; date
  timeout -k 10 400 python bench.py --steps ${STEPS:-4} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/quick.log 2>&1 || { tail -20 gpurun_out/quick.log; exit 1; }
  tail -1 gpurun_out/quick.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, 'sync', round(d['stages_ms']['sync'],3), 'stored/t', d['neighbors_per_particle'])"
fi
