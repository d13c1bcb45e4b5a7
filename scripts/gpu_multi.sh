#!/bin/bash
# Parity tests of several in-tree library variants, then an A/B of their timings:
#   PRE_TESTS="..." VAR_lib_x="tests ..." VAR_lib_y="tests ..." LIBS="lib lib_x lib_y" bash scripts/gpu_multi.sh
# PRE_TESTS run against the default library; every VAR_<lib> against sph-exa_amd/<lib>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${PRE_TESTS:-}" ]; then
  timeout -k 10 500 python -u -m pytest $PRE_TESTS -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pre.log 2>&1
  rc=$?; echo "pre-tests rc=$rc"; tail -4 gpurun_out/pre.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for L in $LIBS; do
  v="VAR_$L"
  T="${!v:-}"
  [ -z "$T" ] && continue
  SPHEXA_AMD_LIB=$PWD/sph-exa_amd/$L/libsphexa_hip.so timeout -k 10 400 python -u -m pytest $T -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/var_$L.log 2>&1
  rc=$?; echo "variant $L tests rc=$rc"; tail -3 gpurun_out/var_$L.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
LIBS="$LIBS" bash scripts/ab_libs.sh
