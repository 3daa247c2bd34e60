# round 4: kman_groups with a 9-bit pass 0 and 5120-item finish regions (three blocks per CU), the round
# path's finish at 5120 items when its regions fit (rfcap: always 8704): every GPU test, the quick bench
# A/B against the previous tree (prev), the world-1 dist line base vs rfcap, phase stamps
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r04c.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r04c.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_gpu_r04c.log
bash tools/ab/gpu_libab.sh r04c 3 prev base xp0 fpf phalf ra4
for v in base rfcap base rfcap; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --no-cpu-baseline > gpurun_out/d1_r04c.json 2> gpurun_out/d1_r04c.err || { tail gpurun_out/d1_r04c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/d1_r04c.json')); print('dist1 $v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config']['stages_ms_per_step_rank0'])"
done
echo "== stamps"
KMAN_LIB=$PWD/kman_amd/lib_ab_stamps/libkman.so timeout -k 10 200 python tools/regionstamps.py uniq 2>&1 | grep -i stamps
echo "== count mode: narrow finish 6 vs 8 waves per SIMD"
BENCH_ARGS="--mode count" bash tools/ab/gpu_libab.sh r04cc 2 base nw8
