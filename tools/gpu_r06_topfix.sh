# round 6: the count finish's top-16-bit sort + run fix-up (k >= ~27):
# parity tests, then config 3 and count -r with it and without (lib_notopfix)
set -e
TAG=${1:-r06tf}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 400 --timeout-method thread -m gpu -x \
  tests/test_gpu_region.py tests/test_gpu_parity.py tests/test_gpu_config3.py tests/test_gpu_canonical.py \
  > gpurun_out/tf_tests_$TAG.log 2>&1 || { tail -60 gpurun_out/tf_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/tf_tests_$TAG.log
for v in on off; do
  if [ $v = off ]; then export KMAN_LIB=$PWD/kman_amd/lib_notopfix/libkman.so; fi
  timeout -k 10 600 python -u tools/widebench.py config3 rc1g --steps 3 > gpurun_out/tf_${TAG}_$v.json 2> gpurun_out/tf_${TAG}_$v.err || { tail -20 gpurun_out/tf_${TAG}_$v.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/tf_${TAG}_$v.json'):
    d = json.loads(l); print('topfix $v', d['line'][:40], round(d['value']/1e9, 2), round(d['ms_per_step'], 2), d.get('rounds', {}).get('kernels_ms_per_step'))"
done
