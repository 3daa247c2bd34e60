# GPU call: rg_extract look-back width A/B (KMAN_RG_XLB = predecessors per lane per round) + PMC traffic
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/xlb_tests.log 2>&1 || { tail -30 gpurun_out/xlb_tests.log; exit 1; }
KMAN_RG_XLB=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_region.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/xlb_tests2.log 2>&1 || { tail -30 gpurun_out/xlb_tests2.log; exit 1; }
tail -1 gpurun_out/xlb_tests2.log
for v in 1 8 1 8; do
  KMAN_RG_XLB=$v timeout -k 10 300 python bench.py --quick --no-cpu-baseline --steps 10 > gpurun_out/xlb_$v.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/xlb_$v.json')); print('$v', round(d['value']/1e9,2), d['config']['stages_ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
for v in 1; do
  KMAN_RG_XLB=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/xlbf_$v -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --quick > /dev/null 2>&1
  python3 - <<PY
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("$R/gpurun_out/xlbf_$v/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE" and "rg_extract" in r["Kernel_Name"]:
            agg["x"].append(float(r["Counter_Value"]))
print("XLB=$v rg_extract FETCH_SIZE KiB/launch", sum(agg["x"]) / max(1, len(agg["x"])))
PY
done
