# one GPU call: every gpu test, the HBM-resident bench line, the world-1 and config-4 dist lines
set -e
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python bench.py --quick --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_quick_$TAG.json 2> gpurun_out/bench_quick_$TAG.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_quick_$TAG.json')); print(d['value']/1e9, d['ms_per_step'], d['config']['stages_ms_per_step'])"
bash tools/gpu_benchdist.sh $TAG
