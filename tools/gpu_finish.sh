set -e
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "finish or sort_stable or extract or command" > gpurun_out/finish_tests.log 2>&1
echo tests-ok
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_split.json 2> gpurun_out/bench_split.err
cat gpurun_out/bench_split.json
