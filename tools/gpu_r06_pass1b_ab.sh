# round 6: pass 1b by chains of 2^m sub-buckets vs one sub-bucket per chain
set -e
TAG=${1:-r06w}
mkdir -p gpurun_out
for one in 0 1; do
  if [ $one = 1 ]; then export KMAN_PASS1B_ONE=1; else unset KMAN_PASS1B_ONE; fi
  timeout -k 10 300 python -u tools/widebench.py grch38u --steps 3 > gpurun_out/p1b_${TAG}_$one.json 2> gpurun_out/p1b_${TAG}_$one.err || { tail -20 gpurun_out/p1b_${TAG}_$one.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/p1b_${TAG}_$one.json').read().strip().splitlines()[-1]); print('one-per-chain $one grch38u', round(d['value']/1e9,2), round(d['ms_per_step'],2), d['rounds']['kernels_ms_per_step'])"
  timeout -k 10 400 python bench.py --dist --mode count --shard-gb 12.5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/p1b_cfg4_${TAG}_$one.json 2> gpurun_out/p1b_cfg4_${TAG}_$one.err || { tail gpurun_out/p1b_cfg4_${TAG}_$one.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/p1b_cfg4_${TAG}_$one.json')); print('one-per-chain $one cfg4', round(d['value']/1e9,2), round(d['ms_per_step'],2), d['config']['stages_ms_per_step_rank0'])"
done
