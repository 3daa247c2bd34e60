# round 5: pass 0's region cursors laid out [segment][bucket] (a wave's 64 cursor adds = 256 contiguous bytes:
# four memory-side atomic requests instead of 64) vs [bucket][segment] (lib_ab_old)
set -e
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_dist_region.py tests/test_gpu_canonical.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05w_tests.log 2>&1 || { tail -40 gpurun_out/r05w_tests.log; exit 1; }
tail -1 gpurun_out/r05w_tests.log
for v in base old base old base old; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --quick --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r05w_q_$v.json 2> gpurun_out/r05w_q_$v.err || { tail -30 gpurun_out/r05w_q_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05w_q_$v.json')); print('c2 $v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config'].get('stages_ms_per_step'))"
done
for v in base old; do
  if [ $v = base ]; then L=$PWD/kman_amd/lib/libkman.so; else L=$PWD/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 python bench.py --gpus 1 --dist --shard-gb 12.5 --mode count --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05w_cfg4_$v.json 2> gpurun_out/r05w_cfg4_$v.err || { tail -30 gpurun_out/r05w_cfg4_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05w_cfg4_$v.json')); print('cfg4 $v', round(d['value']/1e9,2), round(d['ms_per_step'],1), d['config']['stages_ms_per_step_rank0'])"
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r05w_pmcw -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --quick > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r05w_pmcf -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --quick > /dev/null 2>&1
cd $R && python3 tools/pmc_summary.py gpurun_out/r05w_pmcf gpurun_out/r05w_pmcw r05w | grep -E "rg_"
