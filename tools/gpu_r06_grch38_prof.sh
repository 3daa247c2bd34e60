# round 6: rocprofv3 kernel stats of the GRCh38-shaped spectrum line
set -e
TAG=${1:-r06zz}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/gp_$TAG -o run -- python3 $R/tools/widebench.py grch38u --steps 2 > $R/gpurun_out/gp_$TAG.json 2> $R/gpurun_out/gp_$TAG.err
cd $R && head -20 gpurun_out/gp_$TAG/run_kernel_stats.csv
