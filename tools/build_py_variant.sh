#!/usr/bin/env bash
# tools/build_py_variant.sh <name> <python-file> -- libdsm.so from the working tree with the
# python script applied to a scratch copy of csrc/ (it gets the copy's csrc path as argv[1])
# into ab/libdsm_<name>.so (kernel-variant A/B; the edits never touch the tree)
set -e
NAME=$1; PY=$2
T=$(mktemp -d)
cp -r hp-assignment-2_amd/csrc include "$T/"
python3 "$PY" "$T/csrc"
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$T/include ${EXTRA:-}"
$H -c "$T/csrc/dsm_engine.hip" -o "$T/e.o" 2>"$T/warn.txt" || { cat "$T/warn.txt"; exit 1; }
$H -c "$T/csrc/dsm_text.hip" -o "$T/t.o" 2>>"$T/warn.txt" || { cat "$T/warn.txt"; exit 1; }
mkdir -p ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$T/e.o" "$T/t.o" hp-assignment-2_amd/build/dsm_host.o -o "ab/libdsm_$NAME.so"
rm -rf "$T"
echo "ab/libdsm_$NAME.so"
