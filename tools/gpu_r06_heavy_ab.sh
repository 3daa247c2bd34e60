# round 6: what the heavy-key pass 1 costs -- the GRCh38-shaped spectrum line
# with the table and the roomy plan each on and off
set -e
TAG=${1:-r06s}
mkdir -p gpurun_out
for hv in ${HVS:-1 0}; do for rm in ${RMS:-1 0}; do
  KMAN_HEAVY=$hv KMAN_ROOMY=$rm timeout -k 10 300 python -u tools/widebench.py grch38u --steps 3 > gpurun_out/ab_${TAG}_h${hv}r${rm}.json 2> gpurun_out/ab_${TAG}_h${hv}r${rm}.err || { tail -20 gpurun_out/ab_${TAG}_h${hv}r${rm}.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_${TAG}_h${hv}r${rm}.json').read().strip().splitlines()[-1]); print('heavy $hv roomy $rm', round(d['value']/1e9,2), round(d['ms_per_step'],2), d['rounds']['redone_kmers'], d['rounds']['kernels_ms_per_step'])"
done; done
