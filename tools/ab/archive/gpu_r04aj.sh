# pass-0 tile size now that tiles come from the block id: groups path 16 windows per thread (base) vs 12 (ei12, three
# blocks per CU); shard path 12 (base) vs 16 (sei16)
set -e
mkdir -p gpurun_out
for L in ei12 sei16; do
KMAN_LIB=$PWD/kman_amd/lib_ab_$L/libkman.so timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py -q -x -m gpu -k "not slow" --timeout 300 --timeout-method thread > gpurun_out/pytest_r04aj_$L.log 2>&1 || { tail -40 gpurun_out/pytest_r04aj_$L.log; exit 1; }
echo $L tests-ok; tail -1 gpurun_out/pytest_r04aj_$L.log
done
bash tools/ab/gpu_libab.sh r04aj 3 base ei12
for r in 1 2; do for v in base sei16; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/labd_r04aj.json 2> gpurun_out/labd_r04aj.err || { tail gpurun_out/labd_r04aj.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/labd_r04aj.json')); print('dist1 $v', round(d['value']/1e9,2), d['config']['stages_ms_per_step_rank0'])"
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --mode count --shard-gb 12.5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/labc_r04aj.json 2> gpurun_out/labc_r04aj.err || { tail gpurun_out/labc_r04aj.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/labc_r04aj.json')); print('cfg4 $v', round(d['ms_per_step'],1), d['config']['stages_ms_per_step_rank0'])"
done; done
