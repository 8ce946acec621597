cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rb in 0 1 2 4; do echo "== DSOCR_GEMV_RB=$rb"; DSOCR_GEMV_RB=$rb timeout -k 10 120 ./tools/kbench gemv8 || exit 1; done > gpurun_out/kb_gemv.log 2>&1
