# GPU call: region/dist parity after the hot-digit ranks, the bench step, the skewed GRCh38 lines
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_canonical.py tests/test_gpu_dist_region.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r03f_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03f_tests.log; exit 1; }
tail -1 gpurun_out/r03f_tests.log
for m in uniq count; do $T 300 python bench.py --quick --no-cpu-baseline --steps 10 --mode $m > gpurun_out/r03f_bench.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/r03f_bench.json')); print('$m', round(d['value']/1e9,2), d['config']['stages_ms_per_step'])"; done
$T 600 python -u tools/widebench.py grch38s --steps 3 > gpurun_out/r03f_grch38s.json 2> gpurun_out/r03f_grch38s.err
python -c "
import json
for l in open('gpurun_out/r03f_grch38s.json'):
    d=json.loads(l); print(d['line'][:70], round(d['value']/1e9,2), round(d['ms_per_step'],1), json.dumps(d['rounds'].get('phases_ms')))"
