# round 4: the multi-GPU lines at world 1 (1 GB uniq, config 5's canonical count + spectrum, config 4's 12.5 GB
# count shard) and the GRCh38-shaped spectrum line
set -e
TAG=${1:-r04h}
bash tools/gpu_benchdist.sh $TAG
timeout -k 10 500 python -u tools/widebench.py grch38s_spectrum --steps 3 > gpurun_out/g5_$TAG.json 2> gpurun_out/g5_$TAG.err
cat gpurun_out/g5_$TAG.json
