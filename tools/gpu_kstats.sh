# GPU call: rocprofv3 kernel stats of a short bench run (per-kernel averages)
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-k}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ks_$TAG -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --quick > $R/gpurun_out/ks_$TAG.json 2> $R/gpurun_out/ks_$TAG.err
python3 - <<PY
import csv, glob
for f in glob.glob("$R/gpurun_out/ks_$TAG/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        print("%-70s %4s %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
