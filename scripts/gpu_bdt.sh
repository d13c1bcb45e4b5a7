#!/bin/bash
# ve-bdt session: the block time-step parity tests, then the bdt-vs-VE timing at scale; a crash/timeout ends the
# script (test failures do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ve_bdt.py -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/bdt.log 2>&1
rc=$?; tail -15 gpurun_out/bdt.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/bdt_bench.py --side ${BDT_SIDE:-200} --hierarchies 2 > gpurun_out/bdt_bench.log 2>&1
rc=$?; tail -3 gpurun_out/bdt_bench.log
exit $rc
