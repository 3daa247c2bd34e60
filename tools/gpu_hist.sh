# GPU call: spectrum kernel parity + the canonical / dist spectrum tests, then the GRCh38-shaped lines
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hist.py tests/test_gpu_canonical.py tests/test_gpu_dist_region.py -x -q --timeout 300 --timeout-method thread > gpurun_out/hist_tests.log 2>&1 || { tail -40 gpurun_out/hist_tests.log; exit 1; }
tail -1 gpurun_out/hist_tests.log
timeout -k 10 600 python -u tools/widebench.py grch38 --steps 2 > gpurun_out/wide_grch38c.json 2> gpurun_out/wide_grch38c.err
python3 -c "
import json
for l in open('gpurun_out/wide_grch38c.json'):
    d=json.loads(l); print(d['line'], d['value']/1e9, d['ms_per_step'], d['rounds']['phases_ms'])"
