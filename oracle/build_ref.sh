#!/usr/bin/env bash
# oracle/build_ref.sh -- TEST INFRASTRUCTURE ONLY.
# Builds the reference-derived checkers into oracle/_ref/ (git-ignored) from the sources
# where they lie under /root/reference.  No reference text is written into the repository:
# line-range extracts go to a scratch directory that is deleted after compilation.
#   oracle/_ref/cache_simulator_ref    assignment.c compiled unmodified (gcc -O2 -fopenmp)
#   oracle/_ref/ref_lockstep_np4_i32   reference handler text under the lock-step schedule,
#                                      NUM_PROCS=4, MAX_INSTR_NUM=32 (the shipped sizes)
#   oracle/_ref/ref_lockstep_np4_i32_dbg  the same with DEBUG_INSTR (issue-order printf)
#   oracle/_ref/ref_lockstep_np4       NUM_PROCS=4, MAX_INSTR_NUM=4096
#   oracle/_ref/ref_lockstep_np8       NUM_PROCS=8, MAX_INSTR_NUM=4096
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REF="${REF:-/root/reference}"
SRC="$REF/assignment.c"
OUT="$HERE/_ref"
if [ ! -f "$SRC" ]; then echo "build_ref: $SRC absent; skipping" >&2; exit 0; fi
mkdir -p "$OUT"
TMP="$(mktemp -d)"
trap 'rm -rf "$TMP"' EXIT

extract() {  # extract <first> <last> <name> <expected-first-line-regex>
    sed -n "$1,$2p" "$SRC" > "$TMP/$3"
    if ! head -n1 "$TMP/$3" | grep -Eq "$4"; then
        echo "build_ref: $SRC:$1 does not start with /$4/ -- reference changed?" >&2; exit 1
    fi
}
extract 15 81   frag_types.inc   '^typedef unsigned char byte;'
extract 94 115  frag_helpers.inc '^int isBitSet'
extract 177 566 frag_handler.inc 'byte procNodeAddr = msg.address >> 4;'
extract 590 697 frag_issue.inc   'if \(instructionIdx < node.instructionCount - 1\)'
extract 742 773 frag_repl.inc    '^void handleCacheReplacement'
extract 776 822 frag_init.inc    '^void initializeProcessor'
extract 824 876 frag_print.inc   '^void printProcessorState'

CFLAGS="-O2 -w -I$TMP -I$HERE"
gcc $CFLAGS -DNUM_PROCS=4 -DMAX_INSTR_NUM=32   "$HERE/ref_lockstep.c" -o "$OUT/ref_lockstep_np4_i32"
# the reference's own DEBUG_INSTR printf (:595-598) kept: its issue order under the schedule
gcc $CFLAGS -DNUM_PROCS=4 -DMAX_INSTR_NUM=32 -DDEBUG_INSTR "$HERE/ref_lockstep.c" -o "$OUT/ref_lockstep_np4_i32_dbg"
gcc $CFLAGS -DNUM_PROCS=4 -DMAX_INSTR_NUM=4096 "$HERE/ref_lockstep.c" -o "$OUT/ref_lockstep_np4"
gcc $CFLAGS -DNUM_PROCS=8 -DMAX_INSTR_NUM=4096 "$HERE/ref_lockstep.c" -o "$OUT/ref_lockstep_np8"
gcc -O2 -fopenmp "$SRC" -o "$OUT/cache_simulator_ref"
echo "build_ref: built $(ls "$OUT" | tr '\n' ' ')"
