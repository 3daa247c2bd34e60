# rocprofv3 kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE passes of the bench
set -e
R=$GRAFT_REPO_ROOT
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --quick > $R/gpurun_out/prof_$TAG.json 2> $R/gpurun_out/prof_$TAG.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmcf_$TAG -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --quick > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmcw_$TAG -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --quick > /dev/null 2>&1
cd $R && python3 tools/pmc_summary.py gpurun_out/pmcf_$TAG gpurun_out/pmcw_$TAG $TAG uniq 21 1000000000 && cp profiles/pmc_$TAG.json profiles/pmc_current.json gpurun_out/
