# config-4 shard line under an env A/B: gpu_cfg4ab.sh TAG VAR "v1 v2"
set -e
TAG=$1; VAR=$2; VALS=$3
mkdir -p gpurun_out
for v in $VALS; do
  env $VAR=$v timeout -k 10 500 python bench.py --dist --mode count --shard-gb 12.5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4_$TAG.json 2> gpurun_out/c4_$TAG.err || { tail gpurun_out/c4_$TAG.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4_$TAG.json')); print('$VAR=$v cfg4', round(d['value']/1e9,2), round(d['ms_per_step'],1), d['config'].get('stages_ms_per_step_rank0'))"
done
