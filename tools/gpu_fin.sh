# GPU call: region-path parity with the double-buffered finish (KMAN_RG_FIN=2:
# direct global -> LDS loads of the next region), then the A/B against the
# one-block-per-region finish
set -e
mkdir -p gpurun_out
KMAN_RG_FIN=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/fin_tests.log 2>&1 || { tail -40 gpurun_out/fin_tests.log; exit 1; }
tail -1 gpurun_out/fin_tests.log
for v in 2 0 2 0; do
  KMAN_RG_FIN=$v timeout -k 10 300 python bench.py --quick --no-cpu-baseline --steps 10 > gpurun_out/fin_$v.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/fin_$v.json')); print('FIN=$v', round(d['value']/1e9,2), d['config']['stages_ms_per_step'])"
done
