set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/optb2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit 2
FLTEE_BENCH_BACKEND=gloo FLTEE_BENCH_ONE_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 10 --warmup 2 > $O/rehearsal_n2.json 2> $O/rehearsal_n2.err || exit 4
echo done
