cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dots.py -x -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/dots.log 2>&1 && echo "dots ok" >> gpurun_out/rc.log &&
timeout -k 10 600 python bench.py --workload dots2048 --steps 2 --warmup 1 > gpurun_out/benchdots.log 2>&1 && echo "bd ok" >> gpurun_out/rc.log
