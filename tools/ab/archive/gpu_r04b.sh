# round 4: finish block size A/B (512 / 640 / 576 threads for 8-byte items), rg_pass with double-buffered
# counts (pdb), + phase stamps of 512 and 640
set -e
mkdir -p gpurun_out
bash tools/ab/gpu_libab.sh r04b 3 base ft640 ft576 pdb pdb640
for v in stamps stamps640; do
  echo "== $v"
  KMAN_LIB=$PWD/kman_amd/lib_ab_$v/libkman.so timeout -k 10 200 python tools/regionstamps.py uniq 2>&1 | grep -i stamps
done
