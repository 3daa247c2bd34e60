# rg_hist: wave priority 2 while a tile's codes stage (base) vs none (hpr0); dist tests on base first
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_hist.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04as.log 2>&1 || { tail -40 gpurun_out/pytest_r04as.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04as.log
for r in 1 2; do for v in hpr0 base; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/labd_r04as.json 2> gpurun_out/labd_r04as.err || { tail gpurun_out/labd_r04as.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/labd_r04as.json')); print('dist1 $v', round(d['value']/1e9,2), d['config']['stages_ms_per_step_rank0'])"
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --mode count --shard-gb 12.5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/labc_r04as.json 2> gpurun_out/labc_r04as.err || { tail gpurun_out/labc_r04as.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/labc_r04as.json')); print('cfg4 $v', round(d['ms_per_step'],1), d['config']['stages_ms_per_step_rank0'])"
done; done
