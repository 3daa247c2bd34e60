# the multi-GPU pipeline at world size 1 (RCCL self-exchange): dist tests, then the bench per setting
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_dist_region.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 || { tail -40 gpurun_out/dist_tests.log; exit 1; }
tail -1 gpurun_out/dist_tests.log
for cfg in ${CFGS:-KMAN_RG_SMALL=0 KMAN_RG_SMALL=1}; do
  export $cfg
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --dist --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_dist.json 2> gpurun_out/bench_dist.err
  echo "$cfg $(python3 -c 'import json;d=json.loads([l for l in open("gpurun_out/bench_dist.json") if l.startswith("{")][-1]);print(round(d["value"]/1e9,2), d["config"]["stages_ms_per_step"])')"
done | tee gpurun_out/dist1.log
