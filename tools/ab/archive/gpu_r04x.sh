# round-path extraction: current tree (base) vs region.hip before the per-digit output base (s) and before the
# store-loop vmcnt(0) (m0): world-1 1 GB uniq line and config 4's 12.5 GB count shard, stage times
set -e
mkdir -p gpurun_out
for r in 1 2; do for v in base s; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/labd_r04x.json 2> gpurun_out/labd_r04x.err || { tail gpurun_out/labd_r04x.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/labd_r04x.json')); print('dist1 $v', round(d['value']/1e9,2), d['config']['stages_ms_per_step_rank0'])"
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --mode count --shard-gb 12.5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/labc_r04x.json 2> gpurun_out/labc_r04x.err || { tail gpurun_out/labc_r04x.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/labc_r04x.json')); print('cfg4 $v', round(d['ms_per_step'],1), d['config']['stages_ms_per_step_rank0'])"
done; done
