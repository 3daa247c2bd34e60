# SQ counters of one tool run (default: finishbench uniq), two passes of 8 SQ counters.
# usage: gpu_sqpmc.sh TAG [python tool args...]
set -e
R=$GRAFT_REPO_ROOT
TAG=$1; shift
ARGS=${@:-tools/finishbench.py --modes uniq --reps 1}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --kernel-trace --output-format csv -d $R/gpurun_out/sq1_$TAG -o run -- python3 $R/$ARGS > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM --kernel-trace --output-format csv -d $R/gpurun_out/sq2_$TAG -o run -- python3 $R/$ARGS > /dev/null 2>&1
cd $R && python3 tools/sq_summary.py gpurun_out/sq1_$TAG gpurun_out/sq2_$TAG
