# shard tile width by shard size: dist GPU tests, then the world-1 1 GB line and config 4
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_dist.py tests/test_gpu_canonical.py tests/test_gpu_hist.py tests/test_gpu_cli.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_r04ak.log 2>&1 || { tail -40 gpurun_out/pytest_r04ak.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_r04ak.log
bash tools/ab/gpu_r04h.sh r04ak > gpurun_out/r04ak_dist.txt 2>&1
for f in bench_dist1_r04ak bench_cfg5_r04ak bench_cfg4_r04ak; do python3 -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', round(d['value']/1e9,2), round(d['ms_per_step'],1), d['config'].get('stages_ms_per_step_rank0'))"; done
python3 -c "import json; d=json.load(open('gpurun_out/g5_r04ak.json')); print('grch38', d['value']/1e9, d['ms_per_step'])"
