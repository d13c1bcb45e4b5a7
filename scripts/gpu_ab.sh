#!/bin/bash
# Variant check + A/B: parity tests of library LIB (in-tree sph-exa_amd/$LIB), then timing of LIBS.
#   LIB=lib_x TESTS="..." LIBS="lib lib_x" [PRE_TESTS="..."] bash scripts/gpu_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${PRE_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest $PRE_TESTS -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pre.log 2>&1
  echo "pre-tests rc=$?"; tail -4 gpurun_out/pre.log
fi
if [ -n "${TESTS:-}" ]; then
  SPHEXA_AMD_LIB=$PWD/sph-exa_amd/${LIB}/libsphexa_hip.so timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/var.log 2>&1
  rc=$?; echo "variant $LIB tests rc=$rc"; tail -4 gpurun_out/var.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
LIBS="$LIBS" bash scripts/ab_libs.sh
