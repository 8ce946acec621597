cd $GRAFT_REPO_ROOT
bash tools/gpu_session.sh prof1 prof8 profdots
echo "session rc=$?" >> gpurun_out/rc.log
