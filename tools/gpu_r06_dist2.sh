# round 6: dist tests + world-1 lines with the exchange (self part as a
# device copy), sequential and overlapped
set -e
TAG=${1:-r06l}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -x \
  tests/test_gpu_dist.py tests/test_gpu_dist_region.py tests/test_gpu_atsize.py::test_world1_exchange_chunked_messages > gpurun_out/dist_tests_$TAG.log 2>&1 \
  || { tail -60 gpurun_out/dist_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/dist_tests_$TAG.log
cd /tmp
timeout -k 10 300 python3 $R/bench.py --dist --exchange on --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/d1_on_$TAG.json 2> $R/gpurun_out/d1_on_$TAG.err
KMAN_DIST_OVERLAP=1 timeout -k 10 300 python3 $R/bench.py --dist --exchange on --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/d1_ov_$TAG.json 2> $R/gpurun_out/d1_ov_$TAG.err
timeout -k 10 400 python3 $R/bench.py --dist --exchange on --mode count --shard-gb 12.5 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/cfg4_on_$TAG.json 2> $R/gpurun_out/cfg4_on_$TAG.err
KMAN_DIST_OVERLAP=1 timeout -k 10 400 python3 $R/bench.py --dist --exchange on --mode count --shard-gb 12.5 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/cfg4_ov_$TAG.json 2> $R/gpurun_out/cfg4_ov_$TAG.err
cd $R
python3 - <<PY
import json
for n in ("d1_on", "d1_ov", "cfg4_on", "cfg4_ov"):
    d = json.load(open("gpurun_out/%s_$TAG.json" % n)); c = d["config"]
    print(n, round(d["value"] / 1e9, 2), "G/s", round(d["ms_per_step"], 2), "ms", "R", c.get("rounds"), "xch", c.get("exchange"),
          "xch GB/s", c.get("exchange_gbs_rank0"), c.get("stages_ms_per_step_rank0"))
PY
