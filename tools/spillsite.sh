#!/bin/bash
# spillsite.sh FILE.hip MANGLED_SUBSTR [hipcc flags] -- where a kernel spills: the LDS ops / barriers around its scratch stores
src=$1; pat=$2; shift 2
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S "$src" -o /tmp/spill.s "$@" 2>/dev/null
start=$(grep -n "^_Z[^ ]*${pat}[^ ]*:" /tmp/spill.s | head -1 | cut -d: -f1)
awk -v s="$start" 'NR>=s' /tmp/spill.s | awk '/s_endpgm/{print; exit} {print}' > /tmp/spill_k.s
grep -n "scratch_\|s_barrier\|ds_add_rtn\|ds_read\|ds_write\|s_cbranch\|global_load\|global_store" /tmp/spill_k.s | awk '{print $1, $2, $3}' 
