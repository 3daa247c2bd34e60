# GPU call: rocprofv3 kernel stats of the skewed GRCh38 spectrum line (config 5)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
KMAN_DIST_TIMES=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_g5 -o run -- python3 $R/tools/widebench.py grch38s_spectrum --steps 2 > $R/gpurun_out/prof_g5.json 2> $R/gpurun_out/prof_g5.err
cd $R && python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_g5/**/*kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:25]:
    print('%-60s %6s %10.2f ms %9.3f avg' % (r['Name'][:60], r['Calls'], float(r['TotalDurationNs'])/1e6, float(r['AverageNs'])/1e6))
PY
cat gpurun_out/prof_g5.json | cut -c1-400
grep -v "^$" gpurun_out/prof_g5.err | tail -30
