# round 4 measurement call: rocprofv3 kernel stats + FETCH/WRITE PMC passes of the quick bench (profiles/), the SQ
# counters of the bench kernels, the world-1 multi-GPU line with its own PMC passes (pmc_dist_current.json), the
# default bench line (CPU baseline, output, D2H, file-to-file lines)
set -e
TAG=${1:-r04g}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_profile.sh $TAG
python3 - <<PY
import csv, glob
for f in glob.glob("$R/gpurun_out/prof_$TAG/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        print("%-70s %4s %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
bash tools/gpu_sqpmc.sh $TAG tools/regionbench.py uniq 2 > gpurun_out/sq_$TAG.txt 2>&1 || echo "sq pmc failed"
cd /tmp && export TMPDIR=/tmp
WORLD_SIZE=1 timeout -k 10 300 python3 $R/bench.py --dist --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/d1_$TAG.json 2> $R/gpurun_out/d1_$TAG.err
WORLD_SIZE=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/dpmcf_$TAG -o run -- python3 $R/bench.py --dist --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2>&1
WORLD_SIZE=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/dpmcw_$TAG -o run -- python3 $R/bench.py --dist --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2>&1
cd $R && python3 tools/pmc_dist.py gpurun_out/dpmcf_$TAG gpurun_out/dpmcw_$TAG gpurun_out/d1_$TAG.json $TAG && cp profiles/pmc_dist_$TAG.json profiles/pmc_dist_current.json gpurun_out/
timeout -k 10 600 python bench.py > gpurun_out/bench_default_$TAG.json 2> gpurun_out/bench_default_$TAG.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_default_$TAG.json')); print('default', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d['sort_pass_roofline']['frac']); print(json.dumps({k: d.get(k) for k in ('output', 'file_to_file', 'file_to_file_config2', 'pinned_host', 'cpu_baseline')})[:3000])"
