# A/B of an env switch on the HBM-resident bench line: gpu_ab.sh TAG VAR "v1 v2" [rounds] [tests...]
set -e
TAG=$1; VAR=$2; VALS=$3; N=${4:-2}; shift 4 || true
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ab_tests_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/ab_tests_$TAG.log; exit 1; }
  tail -1 gpurun_out/ab_tests_$TAG.log
fi
for r in $(seq $N); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python bench.py --quick --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ab_$TAG.json 2> gpurun_out/ab_$TAG.err || { tail gpurun_out/ab_$TAG.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_$TAG.json')); print('$VAR=$v', round(d['value']/1e9,2), round(d['ms_per_step'],3), d['config']['stages_ms_per_step'], d['roofline'].get('frac'))"
  done
done
