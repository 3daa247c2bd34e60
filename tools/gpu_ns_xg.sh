# A/B: rg_extract look-back chains (KMAN_RG_NS = 64 default, 128, 256) with the XCD-partitioned tickets
set -e
mkdir -p gpurun_out
KMAN_RG_NS=256 timeout -k 10 300 python -u -m pytest tests/test_gpu_region.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ns_tests.log 2>&1 && KMAN_RG_NS=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_region.py -x -q --timeout 200 --timeout-method thread -k groups >> gpurun_out/ns_tests.log 2>&1 || { tail -30 gpurun_out/ns_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/ns_tests.log
st() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], round(d['ms_per_step'],3), d['config']['stages_ms_per_step'])" "$@"; }
for i in 1 2; do
  for x in 64 128 256; do
    KMAN_RG_NS=$x timeout -k 10 200 python bench.py --quick --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ns_$x.json 2> gpurun_out/ns_$x.err
    st gpurun_out/ns_$x.json "ns=$x"
  done
done | tee gpurun_out/ns_ab.log
