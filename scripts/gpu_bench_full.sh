set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bfull
mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
echo done
