# round 6: how pass 1 loses items on the key-ordered GRCh38-shaped line, and
# the new 8-rank heavy-key test
set -e
TAG=${1:-r06z1}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu -x tests/test_gpu_dist_region.py -k "eight_ranks" > gpurun_out/t8_$TAG.log 2>&1 || { tail -30 gpurun_out/t8_$TAG.log; exit 1; }
tail -1 gpurun_out/t8_$TAG.log
KMAN_DROUND_LOG=1 timeout -k 10 400 python -u tools/widebench.py grch38 --steps 1 > gpurun_out/od_$TAG.json 2> gpurun_out/od_$TAG.err || { tail -20 gpurun_out/od_$TAG.err; exit 1; }
grep -E "refit_g|kman_dround_finish" gpurun_out/od_$TAG.err | head -6
