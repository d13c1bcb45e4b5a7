#!/bin/bash
# gravity A/B (fast M2P restructure): gravity tests on the new library, then Evrard n300 steps, lib vs lib_m0
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gravity.py > gpurun_out/r6_grav_tests.log 2>&1 || { tail -20 gpurun_out/r6_grav_tests.log; exit 1; }
tail -2 gpurun_out/r6_grav_tests.log
LIBS="lib lib_m0" ARGS="--init evrard --no-build-step" STEPS=4 WARMUP=2 bash scripts/ab_libs.sh
