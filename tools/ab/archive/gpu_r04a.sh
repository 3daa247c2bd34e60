# round 4, first call: the stripped region path -- every GPU test, the quick
# bench line with the early-count check off / on (A/B), the world-1 dist line
# through bench.py's own spawner
set -e
TAG=${1:-r04a}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_gpu_$TAG.log
bash tools/gpu_ab.sh ${TAG}chk KMAN_RG_CHECK "0 1" 3
timeout -k 10 300 python bench.py --gpus 1 --dist --no-cpu-baseline > gpurun_out/bench_dist1_$TAG.json 2> gpurun_out/bench_dist1_$TAG.err || { tail gpurun_out/bench_dist1_$TAG.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_dist1_$TAG.json')); print('dist1', d['n_gpus'], d['value']/1e9, d['ms_per_step'], d['roofline'], d['config']['stages_ms_per_step_rank0'])"
