# A/B of library builds on the quick bench line: gpu_libab.sh TAG ROUNDS name1 name2 ... (name base = kman_amd/lib)
set -e
TAG=$1; N=$2; shift 2
mkdir -p gpurun_out
for r in $(seq $N); do
  for v in "$@"; do
    if [ "$v" = base ]; then L=kman_amd/lib/libkman.so; else L=kman_amd/lib_ab_$v/libkman.so; fi
    KMAN_LIB=$PWD/$L timeout -k 10 200 python bench.py --quick --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/lab_$TAG.json 2> gpurun_out/lab_$TAG.err || { tail gpurun_out/lab_$TAG.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/lab_$TAG.json')); print('$v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config']['stages_ms_per_step'], round(d['roofline']['frac'],4), round(d['sort_pass_roofline']['frac'],4))"
  done
done
