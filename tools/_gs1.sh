set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_session.sh kernels nocache parity sampling bench bench8
echo "session rc=$?" >> gpurun_out/rc.log
