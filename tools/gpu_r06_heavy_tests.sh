# round 6: the heavy-key / local-redo parity tests and config 5 at size
set -e
TAG=${1:-r06u}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu -x \
  tests/test_gpu_dist_region.py tests/test_gpu_atsize.py -k "heavy or left_out or grch38 or overflow or redo or config5" \
  > gpurun_out/heavy_tests_$TAG.log 2>&1 || { tail -80 gpurun_out/heavy_tests_$TAG.log; exit 1; }
tail -3 gpurun_out/heavy_tests_$TAG.log
