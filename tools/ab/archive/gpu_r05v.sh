# round 5: pass 0 (kman_groups) with 16 / 12 / 8 windows per thread (two / three / four blocks per CU)
set -e
mkdir -p gpurun_out
for e in 12 8; do
  KMAN_EXTRACT_EI=$e timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05v_tests_$e.log 2>&1 || { tail -40 gpurun_out/r05v_tests_$e.log; exit 1; }
  echo "ei $e: $(tail -1 gpurun_out/r05v_tests_$e.log)"
done
for e in 16 12 8 16 12 8; do
  KMAN_EXTRACT_EI=$e timeout -k 10 300 python bench.py --quick --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05v_q_$e.json 2> gpurun_out/r05v_q_$e.err || { tail -30 gpurun_out/r05v_q_$e.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05v_q_$e.json')); print('ei $e', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config'].get('stages_ms_per_step'))"
done
