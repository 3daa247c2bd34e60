# round 5: the two-pass count finish (4-byte items, rest <= 21: the round path's regions) vs three passes
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py tests/test_gpu_dist.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05l_tests.log 2>&1 || { tail -40 gpurun_out/r05l_tests.log; exit 1; }
tail -1 gpurun_out/r05l_tests.log
for v in base notwo base notwo; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --shard-gb 12.5 --mode count --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05l_cfg4_$v.json 2> gpurun_out/r05l_cfg4_$v.err || { tail -30 gpurun_out/r05l_cfg4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05l_cfg4_$v.json')); print('$v', round(d['value']/1e9,2), round(d['ms_per_step'],1), d['config']['rounds'], d['config']['stages_ms_per_step_rank0'])"
done
