# round 4, final tree: every GPU test + smoke, then the measurement call (rocprofv3 stats, PMC, SQ, world-1 line, default bench)
set -e
TAG=${1:-r04r}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
echo tests-ok; tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')"
bash tools/gpu_r04g.sh $TAG
