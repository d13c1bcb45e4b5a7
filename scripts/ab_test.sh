#!/bin/bash
# GPU parity tests of one in-tree library variant, then the A/B timing against others:
#   LIB=lib_x TESTS="tests/test_gpu_parity.py tests/test_gpu_search_builds.py" scripts/ab_test.sh lib lib_x
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SPHEXA_AMD_LIB=$PWD/sph-exa_amd/${LIB:-lib}/libsphexa_hip.so timeout -k 10 ${PYTEST_T:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/ab_test.log 2>&1
rc=$?; tail -3 gpurun_out/ab_test.log
[ $rc -eq 0 ] || exit $rc
[ $# -gt 0 ] && exec_ab=1 && bash scripts/ab_bench.sh "$@"
