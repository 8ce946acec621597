cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
KB_SWZ=1 KB_STAMPS=1 timeout -k 10 120 ./tools/kbench moe1 > gpurun_out/kb.log 2>&1
