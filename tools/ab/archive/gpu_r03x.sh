# EI 16 extraction tiles (single GPU and shard): parity (region, dist, canonical, marked, config 3), bench, config-4 A/B, config-5 lines
set -e
mkdir -p gpurun_out
T="timeout -k 10"
$T 700 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_dist_region.py tests/test_gpu_dist.py tests/test_gpu_canonical.py tests/test_gpu_marked.py tests/test_gpu_config3.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/x_tests.log 2>&1 || { tail -30 gpurun_out/x_tests.log; exit 1; }
tail -1 gpurun_out/x_tests.log
bash tools/gpu_ab.sh x KMAN_RG_EI "16 12" 1
bash tools/gpu_cfg4ab.sh x KMAN_RG_XEI "16 12"
$T 500 python -u tools/widebench.py grch38s_spectrum --steps 3 > gpurun_out/x_g5.json 2> gpurun_out/x_g5.err || { tail gpurun_out/x_g5.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/x_g5.json'):
    d=json.loads(l); print('g5', d.get('line', d.get('metric'))[:40], round(d['value']/1e9,2), round(d['ms_per_step'],1))"
