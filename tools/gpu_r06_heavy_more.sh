set -e
TAG=${1:-r06hm}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -x tests/test_gpu_dist_region.py -k "other_k or eight_ranks" > gpurun_out/hm_$TAG.log 2>&1 || { tail -60 gpurun_out/hm_$TAG.log; exit 1; }
tail -3 gpurun_out/hm_$TAG.log
