# A/B of library builds on the quick bench line: gpu_libab.sh TAG ROUNDS name1 name2 ... (name base = kman_amd/lib)
# every non-base build first passes the region parity tests at k = 21 (else the script stops)
set -e
TAG=$1; N=$2; shift 2
mkdir -p gpurun_out
lib() { if [ "$1" = base ]; then echo $PWD/kman_amd/lib/libkman.so; else echo $PWD/kman_amd/lib_ab_$1/libkman.so; fi; }
for v in "$@"; do
  [ "$v" = base ] && continue
  KMAN_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_region.py -q -x -m gpu -k "matches_oracle and 21" --timeout 120 --timeout-method thread > gpurun_out/lab_par_${TAG}_$v.log 2>&1 || { echo "parity FAILED: $v"; tail -30 gpurun_out/lab_par_${TAG}_$v.log; exit 1; }
  echo "parity ok: $v $(tail -1 gpurun_out/lab_par_${TAG}_$v.log)"
done
for r in $(seq $N); do
  for v in "$@"; do
    KMAN_LIB=$(lib $v) timeout -k 10 200 python bench.py --quick --no-cpu-baseline --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/lab_$TAG.json 2> gpurun_out/lab_$TAG.err || { tail gpurun_out/lab_$TAG.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/lab_$TAG.json')); print('$v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config']['stages_ms_per_step'], round(d['roofline']['frac'],4), round(d['sort_pass_roofline']['frac'],4))"
  done
done
