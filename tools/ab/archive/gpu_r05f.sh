# round 5: compact last pass as its own template instance (no RLE code in it) vs round 4
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py -x -q -m gpu --timeout 120 --timeout-method thread -k "matches_oracle or repeats or full_size or early or pipeline_region" > gpurun_out/r05f_region.log 2>&1 || { tail -40 gpurun_out/r05f_region.log; exit 1; }
tail -1 gpurun_out/r05f_region.log
KMAN_LIB=$PWD/kman_amd/lib_stamps/libkman.so timeout -k 10 200 python tools/regionstamps.py uniq > gpurun_out/r05f_stamps_new.txt 2>&1 || { tail -20 gpurun_out/r05f_stamps_new.txt; exit 1; }
grep "stamps rg_finish" gpurun_out/r05f_stamps_new.txt
bash tools/ab/gpu_libab.sh r05f 3 old base
BENCH_ARGS="--mode count" bash tools/ab/gpu_libab.sh r05fc 1 old base
