cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
KB_STAMPS=1 timeout -k 10 120 ./tools/kbench ${KB_CASES:-attn1 attn8} > gpurun_out/kb.log 2>&1
