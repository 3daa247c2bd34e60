# round 5: the new / changed GPU tests, the full default bench line (CLI phase breakdown, writer-pattern D2H
# probe), the config-4 world-1 line, rocprofv3 per-launch durations of the quick bench beside its HIP events
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_config4.py tests/test_gpu_region.py tests/test_gpu_dist_region.py tests/test_gpu_dist.py -x -q -m gpu --timeout 400 --timeout-method thread -k "config4 or full_size or finish_variants or streamed_rounds or world1 or rccl" > gpurun_out/r05g_tests.log 2>&1 || { tail -40 gpurun_out/r05g_tests.log; exit 1; }
tail -1 gpurun_out/r05g_tests.log
timeout -k 10 600 python bench.py > gpurun_out/r05g_bench.json 2> gpurun_out/r05g_bench.err || { tail -30 gpurun_out/r05g_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05g_bench.json')); print(round(d['value']/1e9,2), d['ms_per_step'], d['config']['stages_ms_per_step']); print(json.dumps(d.get('file_to_file_config2'))[:1500]); print(json.dumps(d.get('output',{}).get('d2h')), d.get('output',{}).get('format_vs_d2h'))"
timeout -k 10 300 python bench.py --gpus 1 --dist --shard-gb 12.5 --mode count --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05g_bench_cfg4.json 2> gpurun_out/r05g_bench_cfg4.err || { tail -30 gpurun_out/r05g_bench_cfg4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05g_bench_cfg4.json')); print(round(d['value']/1e9,2), d['ms_per_step'], d['config']['rccl_ranks'], d['config']['setup_s'], d['config']['stages_ms_per_step_rank0'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05g_kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --quick > $GRAFT_REPO_ROOT/gpurun_out/r05g_kt.json 2> $GRAFT_REPO_ROOT/gpurun_out/r05g_kt.err
cd $GRAFT_REPO_ROOT && python3 tools/kernel_launches.py gpurun_out/r05g_kt gpurun_out/r05g_kt.json > gpurun_out/r05g_launches.json && python3 -c "
import json; d=json.load(open('gpurun_out/r05g_launches.json'))
for k,v in d.items(): print(k, 'rocprof timed avg %.3f min %.3f all %.3f | event %s | ratio %s' % (v['timed_avg_ms'], v['timed_min_ms'], v['all_avg_ms'], v['hip_event_ms'], v['rocprof_over_event']))"
