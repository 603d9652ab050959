set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > $O/bench_full.json 2> $O/bench_full.err || exit 1
FLTEE_BENCH_BACKEND=gloo FLTEE_BENCH_ONE_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 \
  > $O/bench_rehearsal_n2.json 2> $O/bench_rehearsal_n2.err || exit 2
for w in ns c1 c3 c4 c5 mnist30 mnist100; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 bench.py --workload $w --steps 30 --warmup 3 --no-extra --no-cpu-baseline --no-e2e > $O/prof_$w.log 2>&1 || exit 3
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/pmc_fetch.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 10 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > $O/pmc_write.log 2>&1 || exit 5
echo done
