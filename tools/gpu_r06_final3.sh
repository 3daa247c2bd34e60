# round 6 final tree, call C: config 5's GRCh38-shaped and -skewed lines
# (one GPU, widebench: the key rounds with the heavy-key table and the local
# redo), with the round log
set -e
TAG=${1:-r06zz}
mkdir -p gpurun_out
KMAN_DROUND_LOG=1 timeout -k 10 600 python -u tools/widebench.py grch38 --steps 3 > gpurun_out/wide_$TAG.json 2> gpurun_out/wide_$TAG.err || { tail -30 gpurun_out/wide_$TAG.err; exit 1; }
KMAN_DROUND_LOG=1 timeout -k 10 600 python -u tools/widebench.py grch38s_spectrum --steps 3 > gpurun_out/wide_s_$TAG.json 2> gpurun_out/wide_s_$TAG.err || { tail -30 gpurun_out/wide_s_$TAG.err; exit 1; }
python3 - <<PY
import json
for f in ("gpurun_out/wide_$TAG.json", "gpurun_out/wide_s_$TAG.json"):
    for l in open(f):
        d = json.loads(l)
        print(d["line"][:70], round(d["value"] / 1e9, 2), round(d["ms_per_step"], 2), d["rounds"]["redone_kmers"], d["rounds"]["heavy_keys"])
PY
