#!/usr/bin/env bash
# tools/build_text_variant.sh <name> <hipcc flags...> -- libdsm.so with dsm_text.hip rebuilt
# with extra flags (e.g. -DPARSE_OCC=6) into ab/libdsm_<name>.so
set -e
NAME=$1; shift
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude"
T=$(mktemp -d)
$H "$@" -Rpass-analysis=kernel-resource-usage -c hp-assignment-2_amd/csrc/dsm_text.hip -o "$T/t.o" 2>"$T/w.txt"
grep -A10 "parse_kernelILj32E" "$T/w.txt" | grep -E "VGPRs|Occupancy|Spill" | head -4
mkdir -p ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC hp-assignment-2_amd/build/dsm_engine.o "$T/t.o" hp-assignment-2_amd/build/dsm_host.o hp-assignment-2_amd/build/dsm_group.o -L/opt/rocm/lib -lrccl -o "ab/libdsm_$NAME.so"
rm -rf "$T"
echo "ab/libdsm_$NAME.so"
