# narrow count finish: slot reads four at a time (RG_NB) -- k=21 parity on the default build (count and uniq), then A/B in count mode and uniq mode
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04q.log 2>&1 || { tail -40 gpurun_out/pytest_r04q.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04q.log
BENCH_ARGS="--mode count" bash tools/ab/gpu_libab.sh r04q 3 base nb0
bash tools/ab/gpu_libab.sh r04qu 2 base nb0
KMAN_LIB=$PWD/kman_amd/lib_stamps/libkman.so timeout -k 10 300 python tools/regionstamps.py uniq > gpurun_out/stamps_r04q.txt 2>&1; tail -3 gpurun_out/stamps_r04q.txt
KMAN_LIB=$PWD/kman_amd/lib_ab_gp/libkman.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_dist.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04q_gp.log 2>&1 || { tail -30 gpurun_out/pytest_r04q_gp.log; exit 1; }
echo gp-dist-tests-ok; tail -1 gpurun_out/pytest_r04q_gp.log
# round path (world 1 through the spawner): GCAP finish pipelined (gp) vs not (base)
for r in 1 2; do for v in base gp; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --no-cpu-baseline --steps 8 --warmup 2 > gpurun_out/labd_r04q.json 2> gpurun_out/labd_r04q.err || { tail gpurun_out/labd_r04q.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/labd_r04q.json')); print('dist1 $v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config']['stages_ms_per_step_rank0'])"
done; done
