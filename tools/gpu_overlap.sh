# GPU call: multi-GPU tests (SimGroup ranks take the overlapped rounds), then
# the RCCL path at world 1 with the overlapped round forced (async all-to-all
# on the communication stream), A/B against the sequential round
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/ov_tests.log 2>&1 || { tail -40 gpurun_out/ov_tests.log; exit 1; }
tail -1 gpurun_out/ov_tests.log
for v in 1 0 1 0; do
  KMAN_DROUND_MIN_G=1 KMAN_DIST_OVERLAP=$v timeout -k 10 300 python bench.py --dist --no-cpu-baseline --steps 5 > gpurun_out/ov_$v.json 2> gpurun_out/ov_$v.err || { tail -20 gpurun_out/ov_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ov_$v.json')); print('OVERLAP=$v', round(d['value']/1e9,2), round(d['ms_per_step'],2), d['config']['stages_ms_per_step_rank0'])"
done
