# GPU call: region tests, then rg_extract with 256 / 128 / 64 look-back chains (KMAN_RG_NS)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/ns_tests.log 2>&1 || { tail -40 gpurun_out/ns_tests.log; exit 1; }
tail -1 gpurun_out/ns_tests.log
for v in 256 128 64 256 128 64; do
  KMAN_RG_NS=$v timeout -k 10 300 python bench.py --quick --no-cpu-baseline --steps 10 > gpurun_out/ns_$v.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/ns_$v.json')); print('$v', round(d['value']/1e9,2), d['config']['stages_ms_per_step'])"
done
