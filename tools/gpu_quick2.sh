# GPU call: parse + parity tests, then the bench stage times (A/B helper)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py tests/test_gpu_region.py tests/test_gpu_dist_region.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/q2_tests.log 2>&1 || { tail -40 gpurun_out/q2_tests.log; exit 1; }
tail -1 gpurun_out/q2_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --quick --no-cpu-baseline --steps 10 > gpurun_out/q2_bench.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/q2_bench.json')); print(round(d['value']/1e9,2), d['config']['stages_ms_per_step'])"
done
