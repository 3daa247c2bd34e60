# GPU call: the given test files (default: region + dist + parity), fail fast
set -e
mkdir -p gpurun_out
FILES=${@:-tests/test_gpu_region.py tests/test_gpu_dist_region.py tests/test_gpu_parity.py}
timeout -k 10 900 python -u -m pytest $FILES -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/quick.log 2>&1 || { tail -50 gpurun_out/quick.log; exit 1; }
tail -1 gpurun_out/quick.log
