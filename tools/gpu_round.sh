# one GPU call: every gpu test + smoke, the bench lines (HBM-resident, world-1 dist, config 5, config 4), rocprofv3 stats + PMC passes
set -e
TAG=${1:-r03}
bash tools/gpu_tests_bench.sh $TAG
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
bash tools/gpu_profile.sh $TAG
