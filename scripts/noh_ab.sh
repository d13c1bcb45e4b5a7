# Noh -n 300 A/B of skin-search variants selected by environment variables, alternating, twice (same box)
set -o pipefail
mkdir -p gpurun_out/nohab
for i in 1 2; do
  for v in ${VARIANTS:-"SX_SKIN_AUX_PRIO=0" "SX_SKIN_AUX_PRIO=1"}; do
    env $v timeout -k 10 300 python -u bench.py --init noh --side 300 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/nohab/$v.$i.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']['findNeighbors']; print(sys.argv[2], round(d['ms_per_step'],3), 'search', round(sum(k)/len(k),3))" gpurun_out/nohab/$v.$i.json $v
  done
done
