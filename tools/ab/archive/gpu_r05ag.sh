# round 5: persistent pass-0 blocks (XG launches, 16 / 8 windows per thread) loading the next tile's codes behind
# this tile's stores vs one tile per block (KMAN_X_ONE_TILE=1, the same library)
set -e
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_dist_region.py tests/test_gpu_canonical.py tests/test_gpu_dist.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05ag_tests.log 2>&1 || { tail -40 gpurun_out/r05ag_tests.log; exit 1; }
tail -1 gpurun_out/r05ag_tests.log
for v in p one p one p one; do
  if [ $v = one ]; then export KMAN_X_ONE_TILE=1; else unset KMAN_X_ONE_TILE; fi
  timeout -k 10 300 python bench.py --quick --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05ag_q_$v.json 2> gpurun_out/r05ag_q_$v.err || { tail -30 gpurun_out/r05ag_q_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05ag_q_$v.json')); print('c2 $v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config'].get('stages_ms_per_step'))"
done
for v in p one; do
  if [ $v = one ]; then export KMAN_X_ONE_TILE=1; else unset KMAN_X_ONE_TILE; fi
  timeout -k 10 300 python bench.py --gpus 1 --dist --shard-gb 12.5 --mode count --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05ag_cfg4_$v.json 2> gpurun_out/r05ag_cfg4_$v.err || { tail -30 gpurun_out/r05ag_cfg4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05ag_cfg4_$v.json')); print('cfg4 $v', round(d['value']/1e9,2), round(d['ms_per_step'],1), d['config']['stages_ms_per_step_rank0'])"
done
