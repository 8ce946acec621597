cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "moe" > gpurun_out/kern.log 2>&1; echo "kern rc=$?" >> gpurun_out/rc.log
KB_SWZ=1 timeout -k 10 120 ./tools/kbench moe8 > gpurun_out/kb.log 2>&1
timeout -k 10 120 ./tools/kbench moe8 >> gpurun_out/kb.log 2>&1
DSOCR_DN_MM=0 timeout -k 10 120 ./tools/kbench moe8 >> gpurun_out/kb.log 2>&1
