# round 6 final tree, call A: every GPU test, smoke(), the default bench line
# (what the round-end driver runs), in one call
set -e
TAG=${1:-r06zz}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -x --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')"
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['sort_pass_roofline']['frac'], d['cpu_baseline']['value'])"
