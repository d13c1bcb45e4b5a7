#!/bin/bash
# round-6 probes: Noh n300 kernel trace; 2-rank host-transport bench with and without skin lists
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_noh -o run --output-format csv -- python3 -u bench.py --init noh --warmup 3 --steps 10 --no-cpu-baseline > gpurun_out/r6_noh.json 2> gpurun_out/r6_noh.err || exit $?
for sk in 0.08 0; do
  timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29661 bench.py --backend host --side 100 --steps 12 --warmup 2 --skin $sk --no-cpu-baseline > gpurun_out/r6_p2_skin$sk.json 2> gpurun_out/r6_p2_skin$sk.err || exit $?
done
