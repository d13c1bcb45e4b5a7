#!/bin/bash
# Short single-GPU timing run: prints per-kernel times of the default bench workload (no CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/quick.log 2>&1 || { tail -20 gpurun_out/quick.log; exit 1; }
tail -1 gpurun_out/quick.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['kernels_ms'].items()}, 'sync', round(d['stages_ms']['sync'],3))"
