mkdir -p gpurun_out
T="timeout -k 10"
for m in count uniq; do
KMAN_RG_FIN=0 $T 120 python -u tools/finq_cmp.py f0 $m > gpurun_out/finq_f0_$m.log 2>&1; echo "f0 $m rc=$?"
KMAN_RG_FIN=4 $T 120 python -u tools/finq_cmp.py f4 $m > gpurun_out/finq_f4_$m.log 2>&1; echo "f4 $m rc=$?"
KMAN_RG_FIN=4 KMAN_RG_NARROW=0 $T 120 python -u tools/finq_cmp.py f4w $m > gpurun_out/finq_f4w_$m.log 2>&1; echo "f4w $m rc=$?"
done
$T 600 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_vectors.py -q --timeout 120 --timeout-method thread -m gpu -k "multi_gpu or default_raise" > gpurun_out/r03b_tests.log 2>&1
echo "tests rc=$?"; tail -8 gpurun_out/r03b_tests.log
$T 600 python -u -m pytest tests/test_gpu_devformat.py tests/test_gpu_cli.py -q --timeout 120 --timeout-method thread -m gpu -x -k "not multi_gpu" > gpurun_out/r03c_fmt.log 2>&1
echo "fmt tests rc=$?"; tail -3 gpurun_out/r03c_fmt.log
$T 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.err
echo "bench rc=$?"; python -c "import json; d=json.load(open('gpurun_out/r03c_bench.json')); print(d['value']/1e9, json.dumps(d.get('output')))"
