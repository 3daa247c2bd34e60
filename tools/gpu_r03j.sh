# GPU call: round-finish ablations on the skewed GRCh38 spectrum line (rocprof kernel stats)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for d in 1 2 3; do
KMAN_RG_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_g5d$d -o run -- python3 $R/tools/widebench.py grch38s_spectrum --steps 1 > /dev/null 2>&1
python3 - $d <<'PY'
import csv, glob, sys
f = glob.glob('/root/repo/gpurun_out/prof_g5d%s/**/*kernel_stats.csv' % sys.argv[1], recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'rg_finish' in r['Name']: print('dbg', sys.argv[1], r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e6)
PY
done
