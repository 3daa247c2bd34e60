# GPU call: marked extraction placed by an atomic cursor -- marked/round-path parity, skewed GRCh38 lines
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_marked.py tests/test_gpu_dist_region.py tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r03p_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03p_tests.log; exit 1; }
tail -1 gpurun_out/r03p_tests.log
$T 600 python -u tools/widebench.py grch38s --steps 3 > gpurun_out/r03p_wide.json 2> gpurun_out/r03p_wide.err || { tail -20 gpurun_out/r03p_wide.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r03p_wide.json'):
    d=json.loads(l); print(d['line'][:50], round(d['value']/1e9,2), round(d['ms_per_step'],1), json.dumps({k: round(v,1) for k,v in d.get('rounds',{}).get('phases_ms',{}).items()}), d.get('rounds',{}).get('redone_kmers'))"
