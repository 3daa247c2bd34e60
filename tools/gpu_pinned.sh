# GPU call: streamed (pinned-host) tests, then the bench with its pinned-host line
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_region.py -x -q --timeout 300 --timeout-method thread -m gpu -k "streamed or pinned or extract_needs" > gpurun_out/pin_tests.log 2>&1 || { tail -40 gpurun_out/pin_tests.log; exit 1; }
tail -1 gpurun_out/pin_tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/pin_full.json 2>gpurun_out/pin_full.err
python -c "import json; d=json.load(open('gpurun_out/pin_full.json')); print(round(d['value']/1e9,2), json.dumps(d.get('pinned_host')))"
