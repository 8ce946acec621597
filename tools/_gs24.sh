cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bench_dist.py -x -v -m gpu -p no:cacheprovider --timeout 580 --timeout-method thread > gpurun_out/dist.log 2>&1 && echo "dist ok" >> gpurun_out/rc.log
