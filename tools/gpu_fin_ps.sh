# A/B of rg_finish with persistent blocks (KMAN_RG_FIN=3) vs one block per
# region: region / canonical tests with PS on, bench stage times alternating
set -e
mkdir -p gpurun_out
KMAN_RG_FIN=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ps_tests.log 2>&1 || { tail -40 gpurun_out/ps_tests.log; exit 1; }
tail -1 gpurun_out/ps_tests.log
st() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], round(d['ms_per_step'],3), d['config']['stages_ms_per_step'])" "$@"; }
for i in 1 2; do
  for x in 0 3; do
    KMAN_RG_FIN=$x timeout -k 10 200 python bench.py --quick --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ps_$x.json 2> gpurun_out/ps_$x.err
    st gpurun_out/ps_$x.json "fin=$x"
  done
  for x in 0 3; do
    KMAN_RG_FIN=$x timeout -k 10 200 python bench.py --quick --no-cpu-baseline --steps 10 --warmup 3 --mode count > gpurun_out/psc_$x.json 2> gpurun_out/psc_$x.err
    st gpurun_out/psc_$x.json "count fin=$x"
  done
done | tee gpurun_out/ps_ab.log
