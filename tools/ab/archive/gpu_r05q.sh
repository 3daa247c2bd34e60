# round 5: 4-byte count items out of the passes, pending 4-byte items paired into 8-byte stores, vs
# 8-byte items (KMAN_WIDE_ITEMS=1): config 4's rank shape and config 2 in count mode
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py tests/test_gpu_dist.py tests/test_gpu_canonical.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05q_tests.log 2>&1 || { tail -40 gpurun_out/r05q_tests.log; exit 1; }
tail -1 gpurun_out/r05q_tests.log
for v in narrow wide narrow wide; do
  if [ $v = wide ]; then export KMAN_WIDE_ITEMS=1; else unset KMAN_WIDE_ITEMS; fi
  timeout -k 10 300 python bench.py --gpus 1 --dist --shard-gb 12.5 --mode count --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05q_cfg4_$v.json 2> gpurun_out/r05q_cfg4_$v.err || { tail -30 gpurun_out/r05q_cfg4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05q_cfg4_$v.json')); print('cfg4 $v', round(d['value']/1e9,2), round(d['ms_per_step'],1), d['config']['rounds'], d['config']['stages_ms_per_step_rank0'])"
  timeout -k 10 300 python bench.py --quick --mode count --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05q_c2count_$v.json 2> gpurun_out/r05q_c2count_$v.err || { tail -30 gpurun_out/r05q_c2count_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05q_c2count_$v.json')); print('c2count $v', round(d['value']/1e9,2), round(d['ms_per_step'],2), d['config'].get('stages_ms_per_step'))"
done
