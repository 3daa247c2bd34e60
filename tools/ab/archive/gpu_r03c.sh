# early distinct count in the count finish (narrow items): parity + count bench + config-4 shard A/B
set -e
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_dist_region.py tests/test_gpu_canonical.py tests/test_gpu_config3.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/cc_tests.log 2>&1 || { tail -30 gpurun_out/cc_tests.log; exit 1; }
tail -1 gpurun_out/cc_tests.log
for v in 1 0; do
  KMAN_RG_EARLY=$v $T 200 python bench.py --quick --no-cpu-baseline --steps 10 --warmup 3 --mode count > gpurun_out/cc_count.json 2> gpurun_out/cc_count.err || { tail gpurun_out/cc_count.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cc_count.json')); print('count EARLY=$v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config']['stages_ms_per_step'])"
done
bash tools/gpu_cfg4ab.sh cc KMAN_RG_EARLY "1 0"
