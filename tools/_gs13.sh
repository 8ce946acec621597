cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/kall.log 2>&1 && echo "kall ok" >> gpurun_out/rc.log &&
KB_SWZ=1 timeout -k 10 120 ./tools/kbench moe8 > gpurun_out/kb_moe8.log 2>&1 && echo "kb ok" >> gpurun_out/rc.log &&
DSOCR_PARITY_OUT=gpurun_out/parity.jsonl timeout -k 10 600 python -u -m pytest tests/test_full_parity.py -x -q -m gpu -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/par.log 2>&1 && echo "par ok" >> gpurun_out/rc.log &&
timeout -k 10 600 python bench.py --pages-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench8.log 2>&1 && echo "b8 ok" >> gpurun_out/rc.log
