set -e
mkdir -p gpurun_out
for env in "KMAN_RG_FIN=4" "KMAN_RG_FIN=4 KMAN_RG_NARROW=0"; do
  echo "== $env"
  env $env timeout -k 10 300 python -u -m pytest tests/test_gpu_region.py -q --timeout 120 --timeout-method thread -m gpu -k "repeats or overflow or skewed" 2>&1 | tail -4
done
env KMAN_RG_FIN=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_dist_region.py -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -6
