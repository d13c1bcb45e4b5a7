#!/bin/bash
# A/B timing of in-tree library variants: ab_bench.sh lib/dirA lib/dirB ...  (paths relative to sph-exa_amd/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "$@"; do
  echo "== $v"
  SPHEXA_AMD_LIB=$PWD/sph-exa_amd/$v/libsphexa_hip.so bash scripts/quick_bench.sh || exit 1
done
