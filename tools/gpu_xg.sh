# A/B of rg_extract's tickets per XCD partition (KMAN_RG_XG=1) vs one global
# ticket counter: region tests with XG on, bench stage times alternating,
# FETCH / WRITE passes with XG on; then the GRCh38-shaped widebench lines
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
KMAN_RG_XG=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_region.py tests/test_gpu_canonical.py -x -q --timeout 300 --timeout-method thread > gpurun_out/xg_tests.log 2>&1 || { tail -40 gpurun_out/xg_tests.log; exit 1; }
tail -1 gpurun_out/xg_tests.log
st() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], round(d['ms_per_step'],3), d['config']['stages_ms_per_step'])" "$@"; }
for i in 1 2 3; do
  for x in 0 1; do
    KMAN_RG_XG=$x timeout -k 10 200 python bench.py --quick --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/xg_$x.json 2> gpurun_out/xg_$x.err
    st gpurun_out/xg_$x.json "xg=$x"
  done
done | tee gpurun_out/xg_ab.log
cd /tmp && export TMPDIR=/tmp
export KMAN_RG_XG=1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmcf_xg -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --quick > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmcw_xg -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --quick > /dev/null 2>&1
unset KMAN_RG_XG
cd $R && python3 tools/pmc_summary.py gpurun_out/pmcf_xg gpurun_out/pmcw_xg xg uniq 21 1000000000 && cp profiles/pmc_xg.json gpurun_out/
grep -A4 rg_extract gpurun_out/pmc_xg.json || true
timeout -k 10 600 python -u tools/widebench.py grch38 --steps 2 > gpurun_out/wide_grch38.json 2> gpurun_out/wide_grch38.err
cat gpurun_out/wide_grch38.json
