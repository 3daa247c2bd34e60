# GPU call: pass 1b rank A/B (KMAN_RG_1B=1: block-wide atomics) on config 4's shard and the skewed spectrum line
mkdir -p gpurun_out
T="timeout -k 10"
for v in 0 1; do
  KMAN_RG_1B=$v $T 500 python bench.py --dist --mode count --shard-gb 12.5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03r_c4.json 2> gpurun_out/r03r_c4.err || { tail gpurun_out/r03r_c4.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03r_c4.json')); print('1b=$v cfg4', round(d['value']/1e9,2), round(d['ms_per_step'],1), d['config'].get('stages_ms_per_step'))"
  KMAN_RG_1B=$v $T 500 python -u tools/widebench.py grch38s_spectrum --steps 3 > gpurun_out/r03r_g5.json 2> gpurun_out/r03r_g5.err || { tail gpurun_out/r03r_g5.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/r03r_g5.json'):
    d=json.loads(l); print('1b=$v g5', round(d['value']/1e9,2), round(d['ms_per_step'],1), json.dumps({k: round(v,1) for k,v in d.get('rounds',{}).get('phases_ms',{}).items()}))"
done
KMAN_RG_1B=1 $T 600 python -u -m pytest tests/test_gpu_dist_region.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r03r_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03r_tests.log; exit 1; }
tail -1 gpurun_out/r03r_tests.log
