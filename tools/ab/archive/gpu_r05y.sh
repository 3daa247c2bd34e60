# round 5: the 512-thread pass instance (radix <= 256, two blocks per CU) -- pass 1 with pass 0 by 9 bits
# (lib_ab_g9) and pass 1b of the round path -- vs the 1024-thread one (KMAN_PASS_SMALL=0)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_dist.py tests/test_gpu_canonical.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05y_tests.log 2>&1 || { tail -40 gpurun_out/r05y_tests.log; exit 1; }
tail -1 gpurun_out/r05y_tests.log
KMAN_LIB=$PWD/kman_amd/lib_ab_g9/libkman.so timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py -k "full_size or skewed" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05y_tests_g9.log 2>&1 || { tail -40 gpurun_out/r05y_tests_g9.log; exit 1; }
tail -1 gpurun_out/r05y_tests_g9.log
for v in base g9 g9big base g9 g9big; do
  L=$PWD/kman_amd/lib/libkman.so; S=1
  if [ $v = g9 ]; then L=$PWD/kman_amd/lib_ab_g9/libkman.so; fi
  if [ $v = g9big ]; then L=$PWD/kman_amd/lib_ab_g9/libkman.so; S=0; fi
  KMAN_PASS_SMALL=$S KMAN_LIB=$L timeout -k 10 300 python bench.py --quick --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05y_q_$v.json 2> gpurun_out/r05y_q_$v.err || { tail -30 gpurun_out/r05y_q_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05y_q_$v.json')); print('c2 $v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config'].get('stages_ms_per_step'))"
done
for S in 1 0; do
  KMAN_PASS_SMALL=$S timeout -k 10 300 python bench.py --gpus 1 --dist --shard-gb 12.5 --mode count --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05y_cfg4_$S.json 2> gpurun_out/r05y_cfg4_$S.err || { tail -30 gpurun_out/r05y_cfg4_$S.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05y_cfg4_$S.json')); print('cfg4 small=$S', round(d['value']/1e9,2), round(d['ms_per_step'],1), d['config']['stages_ms_per_step_rank0'])"
done
