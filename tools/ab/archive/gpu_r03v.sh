# persistent finish with the next region loaded before the output stores (KMAN_RG_FIN=3): parity + A/B (uniq bench, count)
set -e
mkdir -p gpurun_out
T="timeout -k 10"
KMAN_RG_FIN=3 $T 500 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/v_tests.log 2>&1 || { tail -30 gpurun_out/v_tests.log; exit 1; }
tail -1 gpurun_out/v_tests.log
bash tools/gpu_ab.sh v KMAN_RG_FIN "0 3" 2
for v in 0 3; do
  KMAN_RG_FIN=$v $T 200 python bench.py --quick --no-cpu-baseline --steps 10 --warmup 3 --mode count > gpurun_out/v_count.json 2> gpurun_out/v_count.err || { tail gpurun_out/v_count.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/v_count.json')); print('count FIN=$v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config']['stages_ms_per_step'])"
done
