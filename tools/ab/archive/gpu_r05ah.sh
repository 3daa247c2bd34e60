# round 5: the wide lines on the final tree -- 1 GB count -r, GRCh38-shaped and GRCh38-skewed 3.1 Gbp canonical
# spectra (config 5's output), config 3 (10 GB, k = 31)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/widebench.py rc1g grch38 grch38s_spectrum config3 --steps 3 > gpurun_out/r05ah_wide.json 2> gpurun_out/r05ah_wide.err || { tail -30 gpurun_out/r05ah_wide.err; exit 1; }
python3 -c "
import json
for ln in open('gpurun_out/r05ah_wide.json'):
    d = json.loads(ln); print({k: d[k] for k in d if k not in ('hist_head',)})"
