# round 6: the 0-bit pass 1b as a merge kernel (rg_merge_regions) vs the
# 0-bit rg_pass instance (KMAN_PASS1B_RG=1), after every multi-GPU-path test
set -e
TAG=${1:-r06mg}
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu -x \
  tests/test_gpu_dist_region.py tests/test_gpu_dist.py tests/test_gpu_config4.py tests/test_gpu_cli.py \
  > gpurun_out/mg_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/mg_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/mg_tests_$TAG.log
for v in merge rgpass; do
  if [ $v = rgpass ]; then export KMAN_PASS1B_RG=1; fi
  KMAN_DROUND_P1B=1 timeout -k 10 300 python bench.py --dist --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/mg_${TAG}_$v.json 2> gpurun_out/mg_${TAG}_$v.err || { tail gpurun_out/mg_${TAG}_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/mg_${TAG}_$v.json')); print('$v', round(d['value']/1e9,2), round(d['ms_per_step'],2), d['config']['stages_ms_per_step_rank0'])"
done
