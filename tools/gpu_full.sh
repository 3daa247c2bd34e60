set -e
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo tests-ok; tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_split.json 2> gpurun_out/bench_split.err
cat gpurun_out/bench_split.json
KMAN_LIB=kman_amd/lib_abl4/libkman.so timeout -k 10 300 python tools/finishstamps.py 2>&1 | tail -11
