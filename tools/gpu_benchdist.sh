# GPU call: the multi-GPU pipeline at world 1 (RCCL): 1 GB shard (uniq), config 5's canonical count + spectrum, then config 4's 12.5 GB shard
set -e
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --dist --no-cpu-baseline > gpurun_out/bench_dist1_$TAG.json 2> gpurun_out/bench_dist1_$TAG.err
cat gpurun_out/bench_dist1_$TAG.json
timeout -k 10 300 python bench.py --dist --canonical --mode count --no-cpu-baseline > gpurun_out/bench_cfg5_$TAG.json 2> gpurun_out/bench_cfg5_$TAG.err
cat gpurun_out/bench_cfg5_$TAG.json
timeout -k 10 600 python bench.py --dist --mode count --shard-gb 12.5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg4_$TAG.json 2> gpurun_out/bench_cfg4_$TAG.err
cat gpurun_out/bench_cfg4_$TAG.json
