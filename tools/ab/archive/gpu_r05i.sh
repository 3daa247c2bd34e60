# round 5: the uniq writer cold vs warm in one process
set -e
mkdir -p gpurun_out
FMT_SLICES=1 timeout -k 10 300 python tools/fmtcold.py > gpurun_out/r05i_fmtcold.txt 2>&1 || { tail -20 gpurun_out/r05i_fmtcold.txt; exit 1; }
KMAN_FMT_ZC=1 timeout -k 10 300 python tools/fmtcold.py >> gpurun_out/r05i_fmtcold.txt 2>&1 || { tail -20 gpurun_out/r05i_fmtcold.txt; exit 1; }
KMAN_FMT_ZC=1 timeout -k 10 300 python tools/clibench.py uniq 2 >> gpurun_out/r05i_fmtcold.txt 2>&1 || { tail -20 gpurun_out/r05i_fmtcold.txt; exit 1; }
cat gpurun_out/r05i_fmtcold.txt
