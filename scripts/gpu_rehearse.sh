set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py --steps 20 --no-extra --no-cpu-baseline --no-e2e > gpurun_out/bench_n1_${TAG:-x}.json 2> gpurun_out/bench_n1_${TAG:-x}.err || exit 1
FLTEE_BENCH_BACKEND=gloo FLTEE_BENCH_ONE_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 \
  > gpurun_out/bench_rehearsal_${TAG:-x}.json 2> gpurun_out/bench_rehearsal_${TAG:-x}.err || exit 2
echo done
