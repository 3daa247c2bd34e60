# rg_extract: static XCD-aware tile order by block id (base) vs per-partition ticket atomics (tix); tests on base first
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_dist_region.py tests/test_gpu_canonical.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04ad.log 2>&1 || { tail -40 gpurun_out/pytest_r04ad.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04ad.log
bash tools/ab/gpu_libab.sh r04ad 3 base tix
for v in base tix; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --mode count --shard-gb 12.5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/labc_r04ad.json 2> gpurun_out/labc_r04ad.err || { tail gpurun_out/labc_r04ad.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/labc_r04ad.json')); print('cfg4 $v', round(d['ms_per_step'],1), d['config']['stages_ms_per_step_rank0'])"
done
