set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_canonical.py -x -q --timeout 300 --timeout-method thread > gpurun_out/canon.log 2>&1 || { tail -60 gpurun_out/canon.log; exit 1; }
tail -3 gpurun_out/canon.log
