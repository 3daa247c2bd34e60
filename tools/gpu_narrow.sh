# GPU call: the count finish with 4-byte LDS items (default for count rows
# whose key rest fits 32 bits) through the region / parity / round /
# canonical tests, then an A/B of the count step (KMAN_RG_NARROW=0: 8-byte)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_dist_region.py tests/test_gpu_canonical.py tests/test_gpu_rank_ballot.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/nar_tests.log 2>&1 || { tail -40 gpurun_out/nar_tests.log; exit 1; }
tail -1 gpurun_out/nar_tests.log
for nw in 0 1 0 1; do
  KMAN_RG_NARROW=$nw timeout -k 10 300 python bench.py --quick --no-cpu-baseline --steps 10 --mode count > gpurun_out/nar_bench.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/nar_bench.json')); print('NARROW=$nw count', round(d['value']/1e9,2), d['config']['stages_ms_per_step'])"
done
KMAN_RG_NARROW=0 timeout -k 10 400 python bench.py --dist --mode count --shard-gb 12.5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/nar_cfg4_0.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/nar_cfg4_0.json')); print('cfg4 NARROW=0', round(d['value']/1e9,2), d['config']['stages_ms_per_step_rank0'])"
timeout -k 10 400 python bench.py --dist --mode count --shard-gb 12.5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/nar_cfg4_1.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/nar_cfg4_1.json')); print('cfg4 NARROW=1', round(d['value']/1e9,2), d['config']['stages_ms_per_step_rank0'])"
