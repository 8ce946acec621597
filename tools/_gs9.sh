cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dsq.py -x -v -m gpu -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/dsq.log 2>&1 && echo "dsq ok" >> gpurun_out/rc.log &&
timeout -k 10 600 python bench.py --snapshot q4k --pages-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_q4k8.log 2>&1 && echo "q4k8 ok" >> gpurun_out/rc.log
