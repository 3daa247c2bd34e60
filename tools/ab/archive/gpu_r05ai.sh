# round 5: non-temporal loads of the items (read once) in rg_pass (lib_ab_ntpass) / rg_finish (lib_ab_ntfin)
set -e
mkdir -p gpurun_out
for v in ntpass ntfin; do
  KMAN_LIB=$PWD/kman_amd/lib_ab_$v/libkman.so timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py -k "full_size or matches_oracle" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05ai_tests_$v.log 2>&1 || { tail -40 gpurun_out/r05ai_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r05ai_tests_$v.log)"
done
for v in base ntpass ntfin base ntpass ntfin base ntpass ntfin; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --quick --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05ai_q_$v.json 2> gpurun_out/r05ai_q_$v.err || { tail -30 gpurun_out/r05ai_q_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05ai_q_$v.json')); print('c2 $v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config'].get('stages_ms_per_step'))"
done
