# one GPU call: gpu tests, smoke, bench (with CPU baseline), rocprofv3 stats + PMC passes
set -e
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
cat gpurun_out/bench_$TAG.json
bash tools/gpu_profile.sh $TAG
echo profile-ok
