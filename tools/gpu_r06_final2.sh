# round 6 final tree, call B: rocprofv3 per-launch durations of the quick bench
# beside its HIP events, kernel stats + FETCH/WRITE passes (pmc_<tag>.json),
# the effective clock (GRBM_GUI_ACTIVE), SQ counters of the region kernels,
# the world-1 multi-GPU lines (exchange on: the N > 1 per-rank step) with their
# own FETCH/WRITE passes, config 5's canonical count + spectrum, config 4's shard
set -e
TAG=${1:-r06zz}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt_$TAG -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --quick > $R/gpurun_out/kt_$TAG.json 2> $R/gpurun_out/kt_$TAG.err
cd $R && python3 tools/kernel_launches.py gpurun_out/kt_$TAG gpurun_out/kt_$TAG.json > gpurun_out/launches_$TAG.json
bash tools/gpu_profile.sh $TAG
cd /tmp
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/grbm_$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --quick > /dev/null 2>&1
cd $R && bash tools/gpu_sqpmc.sh $TAG tools/regionbench.py uniq 2 > gpurun_out/sq_$TAG.txt 2>&1 || echo "sq pmc failed"
cd /tmp
WORLD_SIZE=1 timeout -k 10 300 python3 $R/bench.py --dist --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/d1_$TAG.json 2> $R/gpurun_out/d1_$TAG.err
WORLD_SIZE=1 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/dpmcf_$TAG -o run -- python3 $R/bench.py --dist --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2>&1
WORLD_SIZE=1 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/dpmcw_$TAG -o run -- python3 $R/bench.py --dist --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2>&1
cd $R && python3 tools/pmc_dist.py gpurun_out/dpmcf_$TAG gpurun_out/dpmcw_$TAG gpurun_out/d1_$TAG.json $TAG && cp profiles/pmc_dist_$TAG.json profiles/pmc_dist_current.json gpurun_out/
timeout -k 10 300 python bench.py --dist --canonical --mode count --no-cpu-baseline > gpurun_out/bench_cfg5_$TAG.json 2> gpurun_out/bench_cfg5_$TAG.err
timeout -k 10 400 python bench.py --dist --mode count --shard-gb 12.5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg4_$TAG.json 2> gpurun_out/bench_cfg4_$TAG.err
timeout -k 10 400 python bench.py --dist --exchange off --mode count --shard-gb 12.5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_cfg4once_$TAG.json 2> gpurun_out/bench_cfg4once_$TAG.err
python3 - <<PY
import json
d = json.load(open("gpurun_out/launches_$TAG.json"))
for k, v in d.items(): print(k, "rocprof timed avg %.3f | event %s | ratio %s" % (v["timed_avg_ms"], v["hip_event_ms"], v["rocprof_over_event"]))
for n in ("d1", "bench_cfg5", "bench_cfg4", "bench_cfg4once"):
    d = json.load(open("gpurun_out/%s_$TAG.json" % n)); c = d["config"]
    print(n, round(d["value"] / 1e9, 2), round(d["ms_per_step"], 2), c.get("rounds"), c.get("exchange"), c.get("stages_ms_per_step_rank0"))
PY
