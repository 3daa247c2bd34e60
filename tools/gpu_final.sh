# what the round-end driver runs, in one call: every GPU test, smoke(), the
# default bench line
set -e
TAG=${1:-final}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')"
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
