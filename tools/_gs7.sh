cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "moe" > gpurun_out/kern.log 2>&1; echo "kern rc=$?" >> gpurun_out/rc.log
KB_SWZ=1 timeout -k 10 120 ./tools/kbench moe1 > gpurun_out/kb.log 2>&1; echo "kb rc=$?" >> gpurun_out/rc.log
timeout -k 10 120 ./tools/kbench moe1 >> gpurun_out/kb.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_full_parity.py -x -q -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread -s > gpurun_out/par.log 2>&1; echo "par rc=$?" >> gpurun_out/rc.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1; echo "bench rc=$?" >> gpurun_out/rc.log
