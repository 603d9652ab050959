set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_c5 gpurun_out/prof_c3
timeout -k 10 600 python bench.py > gpurun_out/bench_r01d.json 2> gpurun_out/bench_r01d.err || exit 1
# N>1 rehearsal: 2 ranks on cuda:0 over gloo (the driver runs RCCL, one GPU per rank)
FLTEE_BENCH_BACKEND=gloo FLTEE_BENCH_ONE_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 \
  > gpurun_out/bench_rehearsal2.json 2> gpurun_out/bench_rehearsal2.err || exit 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-extra --no-cpu-baseline --no-e2e > gpurun_out/prof_c5.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 bench.py --workload c3 --steps 20 --warmup 2 --no-extra --no-cpu-baseline --no-e2e > gpurun_out/prof_c3.log 2>&1 || exit 4
echo done
