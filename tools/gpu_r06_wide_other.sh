# round 6: the other wide lines (config 3's 10 GB at k = 31; 1 GB count -r)
set -e
TAG=${1:-r06zw}
mkdir -p gpurun_out
for one in 0 1; do
  if [ $one = 1 ]; then export KMAN_PASS1B_ONE=1; else unset KMAN_PASS1B_ONE; fi
  timeout -k 10 600 python -u tools/widebench.py config3 rc1g --steps 3 > gpurun_out/wo_${TAG}_$one.json 2> gpurun_out/wo_${TAG}_$one.err || { tail -20 gpurun_out/wo_${TAG}_$one.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/wo_${TAG}_$one.json'):
    d = json.loads(l); print('one-per-chain $one', d['line'][:40], round(d['value']/1e9, 2), round(d['ms_per_step'], 2), d.get('rounds', {}).get('kernels_ms_per_step'))"
done
