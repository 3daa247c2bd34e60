# round 5: rg_hist -- roll_top + lane-private counter columns (base) vs roll_top + per-wave tables (histwave) vs
# the full roll + lane-private columns (histfull); all three with the next tile prefetched
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_dist.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05n_tests.log 2>&1 || { tail -40 gpurun_out/r05n_tests.log; exit 1; }
tail -1 gpurun_out/r05n_tests.log
for v in base:32 histwave:32 histfull:32 base:32 histwave:32 histfull:32; do
  n=${v%%:*}; gx=${v#*:}
  if [ $n = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$n/libkman.so; fi
  KMAN_HIST_GX=$gx KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --shard-gb 12.5 --mode count --steps 3 --warmup 1 --no-cpu-baseline --no-config4 > gpurun_out/r05n_cfg4_$n$gx.json 2> gpurun_out/r05n_cfg4_$n$gx.err || { tail -30 gpurun_out/r05n_cfg4_$n$gx.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05n_cfg4_$n$gx.json')); print('$v', round(d['value']/1e9,2), round(d['ms_per_step'],1), d['config']['rounds'], d['config']['stages_ms_per_step_rank0'])"
done
