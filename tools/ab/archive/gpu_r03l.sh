# GPU call: per-region stamps of the round finish (diagnostic build): skewed GRCh38 spectrum vs uniform count -r
mkdir -p gpurun_out
export KMAN_LIB=kman_amd/lib_stamps/libkman.so KMAN_RG_STAMPS=1
timeout -k 10 400 python -u tools/widebench.py grch38s_spectrum --steps 1 > gpurun_out/r03l_g5.json 2> gpurun_out/r03l_g5.err || { tail -20 gpurun_out/r03l_g5.err; exit 1; }
grep -A2 "stamps round" gpurun_out/r03l_g5.err | tail -6
timeout -k 10 400 python -u tools/widebench.py rc1g --steps 1 > gpurun_out/r03l_rc.json 2> gpurun_out/r03l_rc.err || { tail -20 gpurun_out/r03l_rc.err; exit 1; }
grep -A2 "stamps round" gpurun_out/r03l_rc.err | tail -6
