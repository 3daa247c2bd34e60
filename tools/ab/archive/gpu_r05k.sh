# round 5: the shard extracted once for all key rounds (one rank): dist parity, config 3 / 4 full-size tests, cfg4 A/B
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_region.py -x -q -m gpu --timeout 300 --timeout-method thread -k "streamed_rounds or overflow or unordered or local_rounds or skewed or canonical or shards_match" > gpurun_out/r05k_tests.log 2>&1 || { tail -40 gpurun_out/r05k_tests.log; exit 1; }
tail -1 gpurun_out/r05k_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_config4.py tests/test_gpu_config3.py -x -q -m gpu --timeout 500 --timeout-method thread > gpurun_out/r05k_full.log 2>&1 || { tail -40 gpurun_out/r05k_full.log; exit 1; }
tail -1 gpurun_out/r05k_full.log
for v in 1 0 1 0; do
  KMAN_DIST_ONCE=$v timeout -k 10 300 python bench.py --gpus 1 --dist --shard-gb 12.5 --mode count --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05k_cfg4_$v.json 2> gpurun_out/r05k_cfg4_$v.err || { tail -30 gpurun_out/r05k_cfg4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05k_cfg4_$v.json')); print('once=$v', round(d['value']/1e9,2), round(d['ms_per_step'],1), d['config']['rounds'], d['config']['stages_ms_per_step_rank0'])"
done
