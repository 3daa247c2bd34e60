# round 5: phase stamps of the region kernels on the final tree (diagnostic build, KMAN_RG_STAMPS)
set -e
mkdir -p gpurun_out
KMAN_LIB=$PWD/kman_amd/lib_stamps/libkman.so timeout -k 10 300 python tools/regionstamps.py uniq > gpurun_out/r05ae_stamps.txt 2>&1 || { tail -20 gpurun_out/r05ae_stamps.txt; exit 1; }
grep stamps gpurun_out/r05ae_stamps.txt
