#!/usr/bin/env bash
# tools/build_base.sh [rev] -- build libdsm.so of git revision `rev` (default HEAD) into
# ab/libdsm_${NAME:-base}.so, for an A/B against the working tree with tools/ab_lib.sh
set -e
REV=${1:-HEAD}
T=$(mktemp -d)
git archive "$REV" hp-assignment-2_amd/csrc include | tar -x -C "$T"
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$T/include"
$H -c "$T/hp-assignment-2_amd/csrc/dsm_engine.hip" -o "$T/e.o" 2>/dev/null
$H -c "$T/hp-assignment-2_amd/csrc/dsm_text.hip" -o "$T/t.o" 2>/dev/null
gcc -O2 -fPIC -std=gnu11 -I"$T/include" -c "$T/hp-assignment-2_amd/csrc/dsm_host.c" -o "$T/h.o"
G=""
if [ -f "$T/hp-assignment-2_amd/csrc/dsm_group.cpp" ]; then   # ABI 5: the RCCL group
  $H -I/opt/rocm/include -c "$T/hp-assignment-2_amd/csrc/dsm_group.cpp" -o "$T/g.o"
  G="$T/g.o -L/opt/rocm/lib -lrccl"
fi
mkdir -p ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$T/e.o" "$T/t.o" "$T/h.o" $G -o ab/libdsm_${NAME:-base}.so
rm -rf "$T"
echo "ab/libdsm_${NAME:-base}.so <- $REV"
