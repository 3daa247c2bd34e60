# GPU call: run-head finish ranks (KMAN_RG_RUNS=1) -- parity, uniform bench and skewed GRCh38 A/B, finish ablations
mkdir -p gpurun_out
T="timeout -k 10"
KMAN_RG_RUNS=1 $T 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r03k_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03k_tests.log; exit 1; }
tail -1 gpurun_out/r03k_tests.log
for h in 0 1; do
  for m in count uniq; do KMAN_RG_RUNS=$h $T 300 python bench.py --quick --no-cpu-baseline --steps 10 --mode $m > gpurun_out/r03k_bench.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/r03k_bench.json')); print('runs=$h $m', round(d['value']/1e9,2), d['config']['stages_ms_per_step'])" || exit 1; done
  KMAN_RG_RUNS=$h $T 600 python -u tools/widebench.py grch38s_spectrum --steps 3 > gpurun_out/r03k_g5_$h.json 2> gpurun_out/r03k_g5_$h.err || exit 1
  python -c "
import json
for l in open('gpurun_out/r03k_g5_$h.json'):
    d=json.loads(l); print('runs=$h', d['line'][:40], round(d['value']/1e9,2), round(d['ms_per_step'],1), json.dumps(d['rounds'].get('phases_ms')))"
done
for d in 1 2 3; do
  KMAN_RG_DBG=$d $T 600 python -u tools/widebench.py grch38s_spectrum --steps 2 > gpurun_out/r03k_g5d.json 2>/dev/null || exit 1
  python -c "
import json
for l in open('gpurun_out/r03k_g5d.json'):
    d=json.loads(l); print('dbg=$d', round(d['ms_per_step'],1), json.dumps(d['rounds'].get('phases_ms')))"
done
