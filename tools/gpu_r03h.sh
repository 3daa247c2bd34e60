# GPU call: hot-digit ranks in pass 0 / 1 on and off (uniform bench, skewed GRCh38 lines)
mkdir -p gpurun_out
T="timeout -k 10"
for h in 0 1; do
  for m in count uniq; do KMAN_RG_HOT=$h $T 300 python bench.py --quick --no-cpu-baseline --steps 10 --mode $m > gpurun_out/r03h_bench.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/r03h_bench.json')); print('hot=$h $m', round(d['value']/1e9,2), d['config']['stages_ms_per_step'])" || exit 1; done
  KMAN_RG_HOT=$h $T 600 python -u tools/widebench.py grch38s --steps 3 > gpurun_out/r03h_grch38s_$h.json 2> gpurun_out/r03h_grch38s_$h.err || exit 1
  python -c "
import json
for l in open('gpurun_out/r03h_grch38s_$h.json'):
    d=json.loads(l); print('hot=$h', d['line'][:40], round(d['value']/1e9,2), round(d['ms_per_step'],1), json.dumps(d['rounds'].get('phases_ms')))"
done
