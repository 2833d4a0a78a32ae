mkdir -p gpurun_out/cfg
for c in hot evict; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu > gpurun_out/cfg/bench_$c.log 2>&1 || exit $?
  echo "$c ok"
done
cd /tmp && export TMPDIR=/tmp; cd - > /dev/null
for c in hot evict; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cfg/kt_$c -o kt -- python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu --no-dump > gpurun_out/cfg/kt_$c.log 2>&1 || exit $?
  echo "kt $c ok"
done
