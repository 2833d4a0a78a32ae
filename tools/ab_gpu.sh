timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 gpurun_out/t.log; [ $rc -le 1 ] || exit $rc
bash tools/ab_lib.sh default abtmp/libdsm_base.so default abtmp/libdsm_base.so
