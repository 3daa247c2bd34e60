# round 6: heavy keys counted apart in pass 1 + left-out regions redone from
# pass 1's output -- parity tests, config 5 at size, the GRCh38-shaped lines
set -e
TAG=${1:-r06n}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -x \
  tests/test_gpu_dist_region.py -k "heavy or left_out or grch38 or streamed or overlapped" \
  > gpurun_out/heavy_tests_$TAG.log 2>&1 || { tail -80 gpurun_out/heavy_tests_$TAG.log; exit 1; }
tail -5 gpurun_out/heavy_tests_$TAG.log
KMAN_DROUND_LOG=1 KMAN_DIST_TIMES=1 timeout -k 10 600 python -u tools/widebench.py grch38 --steps 3 \
  > gpurun_out/wide_$TAG.json 2> gpurun_out/wide_$TAG.err || { tail -40 gpurun_out/wide_$TAG.err; exit 1; }
cat gpurun_out/wide_$TAG.json
timeout -k 10 500 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu -x \
  tests/test_gpu_atsize.py -k config5 --durations=0 > gpurun_out/heavy_atsize_$TAG.log 2>&1 \
  || { tail -60 gpurun_out/heavy_atsize_$TAG.log; exit 1; }
tail -8 gpurun_out/heavy_atsize_$TAG.log
