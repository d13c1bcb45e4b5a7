set -o pipefail
mkdir -p gpurun_out/nohab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_skin.py -s > gpurun_out/nohab/skin.log 2>&1 || { tail -30 gpurun_out/nohab/skin.log; exit 1; }
for i in 1 2; do
  SX_SKIN_SERIAL_EXACT=1 timeout -k 10 300 python -u bench.py --init noh --side 300 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/nohab/serial$i.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --init noh --side 300 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/nohab/early$i.json 2>/dev/null || exit 1
done
