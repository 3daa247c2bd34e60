# count-instance priorities: region/dist tests, the count quick line, config 4 and the world-1 lines
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_dist_region.py tests/test_gpu_canonical.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04an.log 2>&1 || { tail -40 gpurun_out/pytest_r04an.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04an.log
timeout -k 10 300 python bench.py --quick --no-cpu-baseline --mode count --steps 10 --warmup 3 > gpurun_out/lab_r04an.json 2>gpurun_out/lab_r04an.err
python3 -c "import json; d=json.load(open('gpurun_out/lab_r04an.json')); print('count', round(d['value']/1e9,2), d['config']['stages_ms_per_step'])"
bash tools/ab/gpu_r04h.sh r04an > gpurun_out/r04an_dist.txt 2>&1
for f in bench_dist1_r04an bench_cfg5_r04an bench_cfg4_r04an; do python3 -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', round(d['value']/1e9,2), round(d['ms_per_step'],1), d['config'].get('stages_ms_per_step_rank0'))"; done
python3 -c "import json; d=json.load(open('gpurun_out/g5_r04an.json')); print('grch38', d['value']/1e9, d['ms_per_step'])"
