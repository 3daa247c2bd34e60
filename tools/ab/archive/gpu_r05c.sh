# round 5: bucket finish without the PIPE LSD fallback (no VGPR spill) vs round 4; phase stamps of both
set -e
mkdir -p gpurun_out
KMAN_LIB=$PWD/kman_amd/lib_stamps/libkman.so timeout -k 10 200 python tools/regionstamps.py uniq > gpurun_out/r05c_stamps_new.txt 2>&1 || { tail -20 gpurun_out/r05c_stamps_new.txt; exit 1; }
grep stamps gpurun_out/r05c_stamps_new.txt
KMAN_LIB=$PWD/kman_amd/lib_ab_oldst/libkman.so timeout -k 10 200 python tools/regionstamps.py uniq > gpurun_out/r05c_stamps_old.txt 2>&1 || { tail -20 gpurun_out/r05c_stamps_old.txt; exit 1; }
grep stamps gpurun_out/r05c_stamps_old.txt
bash tools/ab/gpu_libab.sh r05c 2 old base
