# GPU call: multi-GPU / round-path parity (incl. the partial redo of
# overflowing regions), then the GRCh38-shaped bench line
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist_region.py tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread -m gpu > gpurun_out/partial_tests.log 2>&1 || { tail -40 gpurun_out/partial_tests.log; exit 1; }
tail -1 gpurun_out/partial_tests.log
KMAN_DIST_TIMES=1 timeout -k 10 600 python -u tools/widebench.py grch38 --steps 2 > gpurun_out/partial_grch38.json 2> gpurun_out/partial_grch38.err || { tail -20 gpurun_out/partial_grch38.err; exit 1; }
cat gpurun_out/partial_grch38.json
