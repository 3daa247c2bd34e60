# GPU call: rocprofv3 kernel stats of the round path: skewed GRCh38 spectrum line and config 4's 12.5 GB shard
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_g5b -o run -- python3 $R/tools/widebench.py grch38s_spectrum --steps 2 > $R/gpurun_out/prof_g5b.json 2> $R/gpurun_out/prof_g5b.err
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4 -o run -- python3 $R/bench.py --dist --mode count --shard-gb 12.5 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_c4.json 2> $R/gpurun_out/prof_c4.err
cd $R && for t in g5b c4; do python3 - $t <<'PY'
import csv, glob, sys
f = glob.glob('gpurun_out/prof_%s/**/*kernel_stats.csv' % sys.argv[1], recursive=True)[0]
rows = list(csv.DictReader(open(f)))
print('==', sys.argv[1])
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print('%-70s %6s %10.2f ms %9.3f avg' % (r['Name'][:70], r['Calls'], float(r['TotalDurationNs'])/1e6, float(r['AverageNs'])/1e6))
PY
done
python3 -c "import json; d=json.load(open('gpurun_out/prof_c4.json')); print(d['value']/1e9, d['ms_per_step'], d['config'].get('stages_ms_per_step'), d['config'].get('rounds'))"
