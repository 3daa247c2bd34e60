# GPU call: region-path parity tests, then an A/B of pass 0 (rg_xown, the
# owned-chain extraction KMAN_RG_OWN=1, vs rg_extract's look-back segments),
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/fin_tests.log 2>&1 || { tail -40 gpurun_out/fin_tests.log; exit 1; }
tail -1 gpurun_out/fin_tests.log
KMAN_RG_OWN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_region.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/fin_tests256.log 2>&1 || { tail -40 gpurun_out/fin_tests256.log; exit 1; }
tail -1 gpurun_out/fin_tests256.log
for v in own256 own old own256 own old; do
  unset KMAN_RG_OWN KMAN_RG_XNT; [ $v != old ] && export KMAN_RG_OWN=1; [ $v = own ] && export KMAN_RG_XNT=512;
  timeout -k 10 300 python bench.py --quick --no-cpu-baseline --steps 10 > gpurun_out/fin_$v.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/fin_$v.json')); print('$v', round(d['value']/1e9,2), d['config']['stages_ms_per_step'])"
done
