#!/usr/bin/env bash
# tools/gpu.sh STEP... -- one GPU session (run it through gpurun) made of named steps, each
# under its own time limit; stops at the first step that faults, aborts or times out
# (rc > 1).  Each step logs to gpurun_out/<name>.log.
#
#   smoke                       __graft_entry__.smoke()
#   tests[:K]                   pytest -m gpu (-k K)
#   bench:CONFIG[:cpu]          bench.py --config CONFIG (--no-cpu unless ":cpu")
#   profile:TAG:CONFIG          tools/profile.sh: kernel trace + SQ / wait / FETCH / WRITE passes
#   kt:TAG:CONFIG               kernel trace only (rocprofv3 --kernel-trace --stats)
#   ab:VAR:V1,V2:N:REPS:DIST    tools/ab_open.py (a knob read at dsm_open, in-process A/B)
#   abl:DIST:N:LIB,LIB          tools/ab_libs.sh (variant builds, "default" = the tree's)
#   util:LIB:DIST               tools/lane_util.py on an instrumented build
#   parse                       GPU text tests, tools/ab_parse.py, tools/prof_parse.sh
#   parsel:LIB,LIB              tools/ab_parse.py per build ("default" = the tree's), twice
#   pipe:N:DIST:PARTS           tools/ab_pipe.py: one engine vs the ensemble in PARTS streams
#   calib                       FETCH_SIZE of a known per-lane 16-B chunk read (ab/calib_fetch)
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {   # step <log name> <seconds> <command...>
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    [ $rc -le 1 ] || exit $rc
}
for s in "$@"; do
    IFS=: read -r kind a b c d e <<< "$s"
    case $kind in
    smoke)   step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    tests)   step "gpu_tests${a:+_$a}" 900 python -u -m pytest tests -m gpu -x -q --timeout 240 \
                 --timeout-method thread ${a:+-k "$a"} ;;
    bench)   if [ "$b" = cpu ]; then step "bench_${a}_cpu" 600 python -u bench.py --config "$a"
             else step "bench_$a" 400 python -u bench.py --config "$a" --no-cpu; fi ;;
    profile) bash tools/profile.sh "$a" --config "$b" --steps 3 --warmup 1 --no-types || exit $? ;;
    kt)      mkdir -p "gpurun_out/prof_$a"
             step "kt_$a" 600 rocprofv3 --kernel-trace --stats --output-format csv \
                 -d "gpurun_out/prof_$a/kt" -o kt -- python3 bench.py --no-cpu --no-types --config "$b" \
                 --steps 3 --warmup 1 ;;
    ab)      step "ab_${a}_${e:-uniform}" 600 python -u tools/ab_open.py "$a" "$b" "${c:-1048576}" "${d:-2}" "${e:-uniform}" ;;
    abl)     step "abl_${a}" 600 bash tools/ab_libs.sh "$a" "$b" ${c//,/ } ;;
    util)    step "util_$b" 300 env DSM_LIB="$a" python -u tools/lane_util.py "$b" ;;
    parse)   step text_tests 600 python -u -m pytest tests/test_gpu_text.py -x -q --timeout 240 --timeout-method thread
             step ab_parse 300 python -u tools/ab_parse.py 65536 5
             bash tools/prof_parse.sh new || exit $? ;;
    parsel)  for r in 1 2; do for L in ${a//,/ }; do
                 if [ "$L" = default ]; then L=""; fi
                 step "parse_${r}_$(basename "${L:-default}" .so)" 300 env DSM_LIB="$L" python -u tools/ab_parse.py 65536 5
             done; done ;;
    pipe)    step "pipe_${b}_$c" 600 python -u tools/ab_pipe.py "$a" 3 "$b" "$c" ;;
    calib)   for cfg in "1048576 64 0" "1048576 64 256" "1048576 8 256" "262144 256 64"; do
                 set -- $cfg
                 d=gpurun_out/calib/l$1_c$2_a$3
                 step "calib_l$1_c$2_a$3" 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$d" \
                     -o calib -- ab/calib_fetch "$1" "$2" "$3"
             done ;;
    *)       echo "tools/gpu.sh: unknown step $s"; exit 2 ;;
    esac
done
exit 0
