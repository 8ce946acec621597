cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --max-new-tokens 64 > gpurun_out/b1_a.log 2>&1 &&
DSOCR_GEMM_FUSED16=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --max-new-tokens 64 > gpurun_out/b1_b.log 2>&1 &&
timeout -k 10 300 python bench.py --pages-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline --max-new-tokens 64 > gpurun_out/b8_a.log 2>&1 &&
DSOCR_GEMM_FUSED16=1 timeout -k 10 300 python bench.py --pages-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline --max-new-tokens 64 > gpurun_out/b8_b.log 2>&1 && echo "ab ok" >> gpurun_out/rc.log
