# round 4: the finish with 768 threads per 8-byte-item region (two blocks per CU, 6 waves per SIMD at 80 VGPRs)
set -e
mkdir -p gpurun_out
KMAN_LIB=$PWD/kman_amd/lib_ab_f768/libkman.so timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_dist_region.py -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/par_r04f.log 2>&1 || { tail -30 gpurun_out/par_r04f.log; exit 1; }
echo "parity f768: $(tail -1 gpurun_out/par_r04f.log)"
bash tools/ab/gpu_libab.sh r04f 3 base f768
echo "== stamps f768"
KMAN_LIB=$PWD/kman_amd/lib_ab_stamps768/libkman.so timeout -k 10 200 python tools/regionstamps.py uniq 2>&1 | grep -i stamps
