# round-path capacity A/B (KMAN_DROUND_PAD): dist tests, config-4 shard line, skewed GRCh38 spectrum line
set -e
mkdir -p gpurun_out
T="timeout -k 10"
$T 500 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_dist.py tests/test_gpu_config3.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pad_tests.log 2>&1 || { tail -30 gpurun_out/pad_tests.log; exit 1; }
tail -1 gpurun_out/pad_tests.log
bash tools/gpu_cfg4ab.sh pad KMAN_DROUND_PAD "1 0"
for v in 1 0; do
  KMAN_DROUND_PAD=$v $T 500 python -u tools/widebench.py grch38s_spectrum --steps 3 > gpurun_out/pad_g5.json 2> gpurun_out/pad_g5.err || { tail gpurun_out/pad_g5.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/pad_g5.json'):
    d=json.loads(l); print('pad=$v g5', round(d['value']/1e9,2), round(d['ms_per_step'],1), json.dumps({k: round(v,1) for k,v in d.get('rounds',{}).get('phases_ms',{}).items()}))"
done
