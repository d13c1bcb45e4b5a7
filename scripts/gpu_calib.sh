#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the access shapes of this library (scripts/fetch_calib.hip): one pass per
# counter, then the factors (known bytes / counter bytes) -> gpurun_out/calib/factors.json (copy to profiles/).
#   hipcc --offload-arch=gfx950 -O3 scripts/fetch_calib.hip -o scripts/fetch_calib   (here, before the call)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/calib
mkdir -p $D
timeout -k 10 120 scripts/fetch_calib > $D/known.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/f -o f -- scripts/fetch_calib > $D/f.log 2>&1 || { tail -5 $D/f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/w -o w -- scripts/fetch_calib > $D/w.log 2>&1 || { tail -5 $D/w.log; exit 1; }
python scripts/fetch_calib.py $D $D/factors.json
