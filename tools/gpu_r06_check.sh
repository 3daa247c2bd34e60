# round 6: after the heavy-key / local-redo change -- every GPU test, the
# default bench line, the world-1 exchange line, the skewed spectrum line
set -e
TAG=${1:-r06p}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -x --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['sort_pass_roofline']['frac'])"
timeout -k 10 600 python bench.py --dist --no-cpu-baseline > gpurun_out/bench_dist1_$TAG.json 2> gpurun_out/bench_dist1_$TAG.err || { tail gpurun_out/bench_dist1_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_dist1_$TAG.json')); print('dist1', d['value']/1e9, d['ms_per_step'], d['config']['stages_ms_per_step_rank0'])"
KMAN_DROUND_LOG=1 timeout -k 10 600 python -u tools/widebench.py grch38s_spectrum --steps 3 > gpurun_out/wide_s_$TAG.json 2> gpurun_out/wide_s_$TAG.err || { tail -30 gpurun_out/wide_s_$TAG.err; exit 1; }
cat gpurun_out/wide_s_$TAG.json
