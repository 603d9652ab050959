set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r1i
mkdir -p $O
FLTEE_BENCH_BACKEND=gloo FLTEE_BENCH_ONE_DEVICE=1 timeout -k 10 900 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 10 --warmup 2 \
  > $O/bench_rehearsal_n4.json 2> $O/bench_rehearsal_n4.err || exit 2
echo done
