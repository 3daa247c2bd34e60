# GPU call: region-path parity tests, then rg_finish A/B (small 256-thread finish
# with 10-bit pass-1 digits vs the big 512-thread finish, KMAN_RG_BIGFIN=1)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/fin_tests.log 2>&1 || { tail -40 gpurun_out/fin_tests.log; exit 1; }
tail -1 gpurun_out/fin_tests.log
for v in small big small big; do
  if [ $v = big ]; then export KMAN_RG_BIGFIN=1; else unset KMAN_RG_BIGFIN; fi
  timeout -k 10 300 python bench.py --quick --no-cpu-baseline --steps 10 > gpurun_out/fin_$v.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/fin_$v.json')); print('$v', round(d['value']/1e9,2), d['config']['stages_ms_per_step'])"
done
