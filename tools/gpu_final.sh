# round-end GPU call: every gpu test + smoke, the default bench line (CPU baseline included), rocprofv3 stats + PMC passes, dist lines, GRCh38-shaped lines
set -e
TAG=${1:-r03}
mkdir -p gpurun_out
bash tools/gpu_tests_bench.sh $TAG
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 300 python bench.py > gpurun_out/bench_default_$TAG.json 2> gpurun_out/bench_default_$TAG.err
python3 -c "import json; d=json.load(open('gpurun_out/bench_default_$TAG.json')); print('default', d['value']/1e9, d['ms_per_step'], d['roofline']['frac'], d.get('cpu_baseline'))"
bash tools/gpu_profile.sh $TAG
timeout -k 10 500 python -u tools/widebench.py grch38s_spectrum --steps 3 > gpurun_out/g5_$TAG.json 2> gpurun_out/g5_$TAG.err
cat gpurun_out/g5_$TAG.json
