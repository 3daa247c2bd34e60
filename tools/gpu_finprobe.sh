# GPU call: rg_finish phase stamps (diagnostic build) + ablations (no sort / no writes)
set -e
mkdir -p gpurun_out
KMAN_LIB=kman_amd/lib_stamps/libkman.so timeout -k 10 300 python tools/regionstamps.py uniq 2>&1 | grep stamps
for d in 0 1 2 3; do
  KMAN_RG_DBG=$d timeout -k 10 300 python bench.py --quick --no-cpu-baseline --steps 10 > gpurun_out/abl_$d.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/abl_$d.json')); print('DBG=$d', d['config']['stages_ms_per_step'])"
done
