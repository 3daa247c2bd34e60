# finish row stores: aligned non-temporal (base) vs unaligned non-temporal (ntun) vs aligned plain (plain); WRITE_SIZE of each
set -e
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/ab/gpu_libab.sh r04s 3 base ntun plain
cd /tmp && export TMPDIR=/tmp
for v in base ntun plain; do
  if [ $v = base ]; then L=$R/kman_amd/lib/libkman.so; else L=$R/kman_amd/lib_ab_$v/libkman.so; fi
  KMAN_LIB=$L timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmcw_r04s_$v -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --quick > /dev/null 2>&1
  python3 - <<PY
import csv, glob, collections
tot = collections.defaultdict(list)
for f in glob.glob("$R/gpurun_out/pmcw_r04s_$v/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "rg_finish" in r["Kernel_Name"]:
            tot[r["Dispatch_Id"]].append(float(r["Counter_Value"]))
vals = [sum(v) for v in tot.values()]
print("$v finish WRITE_SIZE per launch (KiB): " + " ".join("%.0f" % x for x in vals))
PY
done
