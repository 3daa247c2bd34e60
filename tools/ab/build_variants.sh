# build A/B variants of libkman.so: build_variants.sh name1="-DFLAG ..." name2="..."
# each into kman_amd/lib_ab_<name>/libkman.so (scratch builds for gpu_libab.sh)
set -e
cd "$(dirname "$0")/../../kman_amd/csrc"
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  make -s -j8 OUT=../lib_ab_$name EXTRA="$flags" >/dev/null
  echo "built lib_ab_$name ($flags)"
done
