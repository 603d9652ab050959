set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/optb
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/optb/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/optb/pytest.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python -u scripts/bench_sharded_virtual.py > gpurun_out/optb/virtual.jsonl 2> gpurun_out/optb/virtual.err || exit 3
FLTEE_BENCH_BACKEND=gloo FLTEE_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/optb/rehearsal_n2.json 2> gpurun_out/optb/rehearsal_n2.err || exit 4
echo done
