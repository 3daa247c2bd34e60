# GPU call: pass-1b width refitted from the pass-1 counts -- round-path parity, skewed GRCh38 lines, count -r
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_dist.py tests/test_gpu_canonical.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r03m_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03m_tests.log; exit 1; }
tail -1 gpurun_out/r03m_tests.log
$T 600 python -u tools/widebench.py grch38s rc1g --steps 3 > gpurun_out/r03m_wide.json 2> gpurun_out/r03m_wide.err || { tail -20 gpurun_out/r03m_wide.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/r03m_wide.json'):
    d=json.loads(l); print(d['line'][:60], round(d['value']/1e9,2), round(d['ms_per_step'],1), json.dumps(d.get('rounds',{}).get('phases_ms')), d.get('rounds',{}).get('redone_kmers'))"
