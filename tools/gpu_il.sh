# GPU call: chunked pass 0 (kman_groups_begin/_extract/_end) tests, then an
# A/B of the interleaved-chain mapping on the headline step, then the
# pinned-host line with and without the overlap
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/il_tests.log 2>&1 || { tail -40 gpurun_out/il_tests.log; exit 1; }
tail -1 gpurun_out/il_tests.log
for il in 0 1 0 1; do
  KMAN_RG_IL=$il timeout -k 10 300 python bench.py --quick --no-cpu-baseline --steps 10 > gpurun_out/il_bench.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/il_bench.json')); print('IL=$il', round(d['value']/1e9,2), d['config']['stages_ms_per_step'])"
done
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/il_full.json 2>gpurun_out/il_full.err
python -c "import json; d=json.load(open('gpurun_out/il_full.json')); print(json.dumps(d.get('pinned_host')))"
