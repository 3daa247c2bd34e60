# early row count on the round path (uniq with source-rank tags): dist parity + world-1 dist line A/B
set -e
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_dist.py tests/test_gpu_region.py tests/test_gpu_cli.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/yy_tests.log 2>&1 || { tail -30 gpurun_out/yy_tests.log; exit 1; }
tail -1 gpurun_out/yy_tests.log
for r in 1 2; do for v in 1 0; do
  KMAN_RG_EARLY=$v $T 300 python bench.py --dist --no-cpu-baseline > gpurun_out/yy_d1.json 2> gpurun_out/yy_d1.err || { tail gpurun_out/yy_d1.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/yy_d1.json')); print('EARLY=$v dist1', round(d['value']/1e9,2), round(d['ms_per_step'],2), d['config']['stages_ms_per_step_rank0'])"
done; done
