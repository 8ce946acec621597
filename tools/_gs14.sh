cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 && echo "all ok" >> gpurun_out/rc.log &&
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench1.log 2>&1 && echo "b1 ok" >> gpurun_out/rc.log &&
timeout -k 10 600 python bench.py --pages-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench8.log 2>&1 && echo "b8 ok" >> gpurun_out/rc.log
