cd $GRAFT_REPO_ROOT
bash tools/gpu_session.sh dots benchdots gprof
echo "session rc=$?" >> gpurun_out/rc.log
