# round 5: rg_finish -- read-backs and run-length reads unconditional, 8-byte scatter writes without a branch
# (positions past m write a spare slot) vs the committed finish (lib_ab_old)
set -e
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_canonical.py tests/test_gpu_dist_region.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05s_tests.log 2>&1 || { tail -40 gpurun_out/r05s_tests.log; exit 1; }
tail -1 gpurun_out/r05s_tests.log
for v in base old base old base old; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --quick --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05s_q_$v.json 2> gpurun_out/r05s_q_$v.err || { tail -30 gpurun_out/r05s_q_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05s_q_$v.json')); print('c2 $v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config'].get('stages_ms_per_step'))"
done
for v in base old; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --quick --mode count --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05s_c_$v.json 2> gpurun_out/r05s_c_$v.err || { tail -30 gpurun_out/r05s_c_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05s_c_$v.json')); print('c2count $v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config'].get('stages_ms_per_step'))"
done
