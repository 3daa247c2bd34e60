# GPU call: region-path parity with the pipelined finish (KMAN_RG_FIN=4),
# then an alternating A/B of the bench step against the default finish
set -e
mkdir -p gpurun_out
KMAN_RG_FIN=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_dist_region.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/finq_tests.log 2>&1 || { tail -40 gpurun_out/finq_tests.log; exit 1; }
tail -1 gpurun_out/finq_tests.log
for v in 4 0 4 0; do
  KMAN_RG_FIN=$v timeout -k 10 300 python bench.py --quick --no-cpu-baseline --steps 10 > gpurun_out/finq_$v.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/finq_$v.json')); print('FIN=$v', round(d['value']/1e9,2), d['config']['stages_ms_per_step'])"
done
