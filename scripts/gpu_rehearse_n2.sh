# gpurun job: rehearse bench.py --gpus 2 on a 1-GPU box (gloo, both ranks on cuda:0):
# first with a tiny extras budget (the watchdog path), then in full
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-n2}
mkdir -p $OUT
export FLTEE_BENCH_BACKEND=gloo FLTEE_BENCH_ONE_DEVICE=1
# (the watchdog leg ends with status 3 by design when the budget cuts a leg short: the
# headline line is printed, and a stuck leg must not read as success)
FLTEE_BENCH_EXTRA_BUDGET_S=${BUDGET1:-8} timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 > $OUT/watchdog.json 2> $OUT/watchdog.err
rc=$?
echo "watchdog leg rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 3 ]; then tail -20 $OUT/watchdog.err; exit 11; fi
tail -c 400 $OUT/watchdog.json; echo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 2 > $OUT/full.json 2> $OUT/full.err || { echo "rc=$?"; tail -20 $OUT/full.err; exit 12; }
tail -c 600 $OUT/full.json; echo
