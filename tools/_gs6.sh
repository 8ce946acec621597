cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -x > gpurun_out/gpu_all.log 2>&1; echo "gpu_all rc=$?" >> gpurun_out/rc.log
