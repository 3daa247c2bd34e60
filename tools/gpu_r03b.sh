# GPU call (round 3): multi-GPU CLI at world 1 + vectors default; the
# pipelined finish (KMAN_RG_FIN=4) on the round path, narrow and wide items
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_vectors.py -q --timeout 120 --timeout-method thread -m gpu -k "multi_gpu or default_raise" > gpurun_out/r03b_tests.log 2>&1
echo "tests rc=$?"; tail -8 gpurun_out/r03b_tests.log
for env in "KMAN_RG_FIN=4" "KMAN_RG_FIN=4 KMAN_RG_NARROW=0"; do
  echo "== $env"
  env $env $T 300 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -12
done
