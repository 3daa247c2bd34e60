# round 6: pass 1b with 0 bits (merge + source tag only) when a (b, d) region
# fits -- every multi-GPU-path test, then the world-1 uniq line with pass 1b
# forced as N > 1 runs it: the new plan (KMAN_DROUND_P1B=1) vs the old one's
# g = 1 (KMAN_DROUND_MIN_G=1)
set -e
TAG=${1:-r06p0}
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu -x \
  tests/test_gpu_dist_region.py tests/test_gpu_dist.py tests/test_gpu_config4.py tests/test_gpu_cli.py \
  > gpurun_out/p0_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/p0_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/p0_tests_$TAG.log
for v in P1B MIN_G; do
  env KMAN_DROUND_$v=1 timeout -k 10 300 python bench.py --dist --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/p0_${TAG}_$v.json 2> gpurun_out/p0_${TAG}_$v.err || { tail gpurun_out/p0_${TAG}_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/p0_${TAG}_$v.json')); print('$v', round(d['value']/1e9,2), round(d['ms_per_step'],2), d['config']['stages_ms_per_step_rank0'])"
done
