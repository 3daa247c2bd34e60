# SQ counters of the region kernels for two library builds: gpu_sq_ab.sh TAG name1 name2 (base = kman_amd/lib)
set -e
R=$GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p $R/gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then L=$R/kman_amd/lib/libkman.so; else L=$R/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L bash $R/tools/gpu_sqpmc.sh ${TAG}_$v tools/regionbench.py uniq 2 > $R/gpurun_out/sq_${TAG}_$v.txt 2>&1 || { echo "sq failed $v"; exit 1; }
  echo "== $v"; grep -A 17 "rg_finish" $R/gpurun_out/sq_${TAG}_$v.txt | head -18
done
