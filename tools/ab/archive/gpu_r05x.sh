# round 5: pass 0 by 9 bits (512 buckets) + pass 1 by 8 (lib_ab_g9) vs 8 + 9, now that the cursor adds are cheap
set -e
mkdir -p gpurun_out
KMAN_LIB=$PWD/kman_amd/lib_ab_g9/libkman.so timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py -k "full_size or skewed" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05x_tests.log 2>&1 || { tail -40 gpurun_out/r05x_tests.log; exit 1; }
tail -1 gpurun_out/r05x_tests.log
for v in base g9 base g9 base g9; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --quick --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05x_q_$v.json 2> gpurun_out/r05x_q_$v.err || { tail -30 gpurun_out/r05x_q_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05x_q_$v.json')); print('c2 $v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config'].get('stages_ms_per_step'))"
done
