# one GPU call: every gpu test, smoke, bench (N=1 and the N>1 code path at world 1)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
timeout -k 10 300 python bench.py --dist --no-cpu-baseline > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.err
cat gpurun_out/bench_dist1.json
