#!/usr/bin/env bash
# full GPU round at HEAD, then C4's budget (DSM_FF_BUDGET_ROUNDS) with the plain budget pass
bash tools/gpu_round.sh || exit $?
timeout -k 10 500 python -u tools/ab_open.py DSM_FF_BUDGET_ROUNDS 384,256,512,768,1024 1048576 2 hot > gpurun_out/ab_p0.log 2>&1
echo done
