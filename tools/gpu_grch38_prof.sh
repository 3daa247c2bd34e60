# rocprofv3 kernel stats of the GRCh38-shaped lines (where the key rounds' time goes on skewed canonical keys)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_grch38 -o run -- python3 $R/tools/widebench.py grch38 --steps 1 > $R/gpurun_out/prof_grch38.json 2> $R/gpurun_out/prof_grch38.err
cd $R && python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_grch38/run_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print("%-70s %5s %10.3f ms total %8.3f ms avg" % (r["Name"][:70], r["Calls"], float(r["TotalDurationNs"]) / 1e6,
                                                       float(r["AverageNs"]) / 1e6))
PY
