# config 4 again, alternating: extract priorities (base) vs none (xp0)
set -e
mkdir -p gpurun_out
for r in 1 2; do for v in xp0 base; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --mode count --shard-gb 12.5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/labc_r04aq.json 2> gpurun_out/labc_r04aq.err || { tail gpurun_out/labc_r04aq.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/labc_r04aq.json')); print('cfg4 $v', round(d['ms_per_step'],1), d['config']['stages_ms_per_step_rank0'])"
done; done
