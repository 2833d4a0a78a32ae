#!/usr/bin/env bash
# tools/build_variant.sh <name> <sed-expr> [<sed-expr> ...] -- build libdsm.so from the
# working tree with sed edits applied to csrc/dsm_engine.hip into ab/libdsm_<name>.so
# (kernel-variant A/B with tools/ab_lib.sh; the edits never touch the tree)
set -e
NAME=$1; shift
T=$(mktemp -d)
cp -r hp-assignment-2_amd/csrc include "$T/"
for e in "$@"; do sed -i "$e" "$T/csrc/${FILE:-dsm_engine.hip}"; done
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$T/include ${EXTRA:-}"
$H -c "$T/csrc/dsm_engine.hip" -o "$T/e.o" 2>"$T/warn.txt" || { cat "$T/warn.txt"; exit 1; }
grep -i "spill\|occupancy" "$T/warn.txt" | head -5 || true
mkdir -p ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$T/e.o" hp-assignment-2_amd/build/dsm_text.o hp-assignment-2_amd/build/dsm_host.o hp-assignment-2_amd/build/dsm_group.o -L/opt/rocm/lib -lrccl -o "ab/libdsm_$NAME.so"
rm -rf "$T"
echo "ab/libdsm_$NAME.so"
