# round 4: config 4's per-rank shape (12.5 GB, count, world 1) across library builds
set -e
mkdir -p gpurun_out
for v in "$@"; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 500 python bench.py --dist --mode count --shard-gb 12.5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4_r04d.json 2> gpurun_out/c4_r04d.err || { tail gpurun_out/c4_r04d.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4_r04d.json')); print('cfg4 $v', round(d['value']/1e9,2), round(d['ms_per_step'],1), d['config'].get('stages_ms_per_step_rank0'), d['config'].get('rounds'))"
done
