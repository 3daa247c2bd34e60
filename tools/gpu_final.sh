# one GPU call: every gpu test, smoke, the default bench line (N = 1, with the CPU baseline)
set -e
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
echo smoke-ok
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value']/1e9, d['ms_per_step'], d['config']['stages_ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'])"
