# round 5: the bucket finish against round 4's LSD finish on the quick bench line (3 alternating rounds)
set -e
mkdir -p gpurun_out
bash tools/ab/gpu_libab.sh r05b 3 old base
