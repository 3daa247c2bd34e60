# GPU call (round 3): the new word-key path, the multi-GPU CLI at world 1,
# the RCCL exchange tests, and the pipelined finish's failing case
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cli.py tests/test_gpu_canonical.py tests/test_gpu_devformat.py tests/test_gpu_dist.py tests/test_gpu_vectors.py -q --timeout 120 --timeout-method thread -m gpu -k "wide or command_matches or cli or canonical or devformat or dist or vectors" > gpurun_out/r03a_tests.log 2>&1
echo "tests rc=$?"
tail -30 gpurun_out/r03a_tests.log
KMAN_RG_FIN=4 $T 300 python -u -m pytest tests/test_gpu_region.py -q --timeout 120 --timeout-method thread -m gpu -k "repeats or overflow or skewed" > gpurun_out/r03a_finq.log 2>&1
echo "finq rc=$?"
tail -15 gpurun_out/r03a_finq.log
