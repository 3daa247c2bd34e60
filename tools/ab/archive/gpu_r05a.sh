# round 5: the bucket finish (region parity incl. the forced-LSD fallback), then old vs new on the quick bench line
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r05a_region.log 2>&1 || { tail -40 gpurun_out/r05a_region.log; exit 1; }
tail -1 gpurun_out/r05a_region.log
KMAN_RG_LSD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py -x -q -m gpu --timeout 120 --timeout-method thread -k "matches_oracle or repeats or full_size" > gpurun_out/r05a_region_lsd.log 2>&1 || { tail -40 gpurun_out/r05a_region_lsd.log; exit 1; }
tail -1 gpurun_out/r05a_region_lsd.log
bash tools/ab/gpu_libab.sh r05a 3 old base
