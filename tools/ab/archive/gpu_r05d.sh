# round 5: bucket finish, reads back to back (levels), vs round 4: region parity (+ forced LSD), stamps, A/B uniq + count
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py -x -q -m gpu --timeout 120 --timeout-method thread -k "matches_oracle or repeats or full_size or early" > gpurun_out/r05d_region.log 2>&1 || { tail -40 gpurun_out/r05d_region.log; exit 1; }
tail -1 gpurun_out/r05d_region.log
KMAN_LIB=$PWD/kman_amd/lib_stamps/libkman.so timeout -k 10 200 python tools/regionstamps.py uniq > gpurun_out/r05d_stamps_new.txt 2>&1 || { tail -20 gpurun_out/r05d_stamps_new.txt; exit 1; }
grep "stamps rg_finish" gpurun_out/r05d_stamps_new.txt
bash tools/ab/gpu_libab.sh r05d 2 old base
BENCH_ARGS="--mode count" bash tools/ab/gpu_libab.sh r05dc 1 old base
