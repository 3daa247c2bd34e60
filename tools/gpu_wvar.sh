# rg_pass write-phase variants (RG_WVAR builds in kman_amd/lib_abl_w*): stage times
set -e
mkdir -p gpurun_out
for v in ${@:-w0 w1 w2 w3 w4 w5}; do
  echo "== RG_WVAR=$v"
  KMAN_LIB=kman_amd/lib_abl_$v/libkman.so timeout -k 10 150 python -u tools/regionbench.py uniq 0,0,0
done 2>&1 | tee gpurun_out/wvar.log
