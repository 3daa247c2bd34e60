# rg_extract: wave priority 2 while a tile's codes load and its items store, 0 for the roll/rank (base) vs none (xp0)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04ap.log 2>&1 || { tail -40 gpurun_out/pytest_r04ap.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04ap.log
bash tools/ab/gpu_libab.sh r04ap 3 base xp0
for v in base xp0; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --mode count --shard-gb 12.5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/labc_r04ap.json 2> gpurun_out/labc_r04ap.err || { tail gpurun_out/labc_r04ap.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/labc_r04ap.json')); print('cfg4 $v', round(d['ms_per_step'],1), d['config']['stages_ms_per_step_rank0'])"
done
