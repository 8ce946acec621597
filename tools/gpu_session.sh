#!/bin/bash
# GPU session runner for gpurun: each step bounded by its own timeout; test failures
# (pytest rc=1) do not stop the session, anything else (fault, abort, timeout) does.
# usage: tools/gpu_session.sh <step>...   steps: kernels model_tiny model_full smoke bench bench_prof
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; echo "rc=$rc :: $*" >> gpurun_out/rc.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; return 0; }
for step in "$@"; do
  case $step in
    kernels) run 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/kernels.log 2>&1 ;;
    model_tiny) run 600 python -m pytest tests/test_gpu_model.py -q -m gpu -rf -p no:cacheprovider --timeout 300 --timeout-method thread -k "tiny or eos or mask or safetensors" > gpurun_out/model_tiny.log 2>&1 ;;
    model_full) run 900 python -m pytest tests/test_gpu_model.py -q -m gpu -rf -p no:cacheprovider --timeout 300 --timeout-method thread -k "full" > gpurun_out/model_full.log 2>&1 ;;
    parity) DSOCR_PARITY_OUT=gpurun_out/parity.jsonl run 900 python -u -m pytest tests/test_full_parity.py -q -m gpu -rf -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/parity.log 2>&1 ;;
    nocache) run 600 python -u -m pytest tests/test_gpu_model.py -q -m gpu -rf -p no:cacheprovider --timeout 300 --timeout-method thread -k "without_cache or stream" > gpurun_out/nocache.log 2>&1 ;;
    sampling) run 600 python -u -m pytest tests/test_sampling.py -q -m gpu -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/sampling.log 2>&1 ;;
    bench8) run 900 python bench.py --pages-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench8.log 2>&1 ;;
    gprof) run 600 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof -o g --output-format csv -- python bench.py --steps 1 --warmup 0 --max-new-tokens 32 --no-cpu-baseline --roofline-iters 4 > gpurun_out/gprof.log 2>&1 ;;
    gprof8) run 600 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof8 -o g --output-format csv -- python bench.py --pages-per-gpu 8 --steps 1 --warmup 0 --max-new-tokens 32 --no-cpu-baseline --roofline-iters 4 > gpurun_out/gprof8.log 2>&1 ;;
    dots) run 900 python -u -m pytest tests/test_dots.py -q -m gpu -rf -p no:cacheprovider --timeout 600 --timeout-method thread -s > gpurun_out/dots.log 2>&1 ;;
    benchdots) run 900 python bench.py --workload dots2048 --steps 2 --warmup 1 > gpurun_out/benchdots${TAG:+_$TAG}.log 2>&1 ;;
    prof1) DSOCR_NO_GRAPH=1 run 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o b1 --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1 ;;
    prof8) DSOCR_NO_GRAPH=1 run 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o b8 --output-format csv -- python bench.py --pages-per-gpu 8 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof8.log 2>&1 ;;
    profdots) run 900 rocprofv3 --kernel-trace --stats -d gpurun_out/profdots -o dots --output-format csv -- python bench.py --workload dots2048 --steps 1 --warmup 1 > gpurun_out/profdots.log 2>&1 ;;
    # round-6 switch table: every DSOCR_* switch A/B'd in separate processes on one box
    abv) run 900 tools/env_ab_vision.sh base: attn_fwd2:DSOCR_ATTN_SPLIT=0 one_stream:DSOCR_VIS_STREAMS=0 nst2:DSOCR_GEMM_NST=2 group1:DSOCR_GEMM_GROUP_M=1 no_ksplit:DSOCR_ATTN_KSPLIT=0 > gpurun_out/abv.log 2>&1 ;;
    abd1) AB_TOKENS=256 AB_ROUNDS=2 run 900 tools/env_ab.sh base: qkv_sep:DSOCR_QKV_ATTN=0 screen0:DSOCR_SCREEN=0 gu_order0:DSOCR_GU_ORDER=0 kvdelay0:DSOCR_ATT_KV_DELAY=0 persist:DSOCR_PERSIST=1 no_graph:DSOCR_NO_GRAPH=1 > gpurun_out/abd1.log 2>&1 ;;
    abd8) AB_TOKENS=128 AB_ROUNDS=2 AB_EXTRA="--pages 8 --text-pages" run 900 tools/env_ab.sh base: route0:DSOCR_ROUTE_FUSED=0 mmswz0:DSOCR_MM_SWZ=0 routerswz0:DSOCR_ROUTER_SWZ=0 guks1:DSOCR_GU_KS=1 guks4:DSOCR_GU_KS=4 dnks1:DSOCR_DN_KS=1 > gpurun_out/abd8.log 2>&1 ;;
    katt_split) run 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "test_attention" > gpurun_out/katt_split.log 2>&1 ;;
    # two library builds of the same tree (tools/prof_vision.py --lib), alternating processes
    vab) for i in 1 2; do for L in dsocr_ab_old dsocr; do echo "== $L" >> gpurun_out/vab.log; run 180 python tools/prof_vision.py --reps 4 --lib deepseek-ocr.rs_amd/lib/lib$L.so >> gpurun_out/vab.log 2>&1; done; done ;;
    vprof) run 300 rocprofv3 --kernel-trace --stats -d gpurun_out/vprof -o v --output-format csv -- python tools/prof_vision.py --reps 3 > gpurun_out/vprof.log 2>&1 ;;
    dab) for i in 1 2; do for L in dsocr_ab_old dsocr; do echo "== $L" >> gpurun_out/dab.log; run 180 python tools/ab_trace.py --tokens 256 --rounds 2 --variant "$L:" --out gpurun_out/dab_$L.json --lib deepseek-ocr.rs_amd/lib/lib$L.so ${AB_EXTRA} >> gpurun_out/dab.log 2>&1; done; done ;;
    gu_ab) AB_TOKENS=256 AB_ROUNDS=2 run 900 tools/env_ab.sh base: gu0:DSOCR_GU_ORDER=0 base: gu0:DSOCR_GU_ORDER=0 base: gu0:DSOCR_GU_ORDER=0 > gpurun_out/gu_ab.log 2>&1 ;;
    bgu) for i in 1 2; do for o in 1 0; do echo "== GU_ORDER=$o" >> gpurun_out/bgu.log; DSOCR_GU_ORDER=$o run 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-chain-roofline --roofline-iters 4 >> gpurun_out/bgu.log 2>&1; done; done ;;
    kdots) run 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention_bf16" > gpurun_out/kdots.log 2>&1 ;;
    dpp) for i in 1 2; do for v in 0 1; do echo "== DOTS_ATTN_PP=$v" >> gpurun_out/dpp.log; DSOCR_DOTS_ATTN_PP=$v run 300 python bench.py --workload dots2048 --steps 2 --warmup 1 >> gpurun_out/dpp.log 2>&1; done; done ;;
    rpb_ab) AB_TOKENS=256 AB_ROUNDS=2 run 900 tools/env_ab.sh base: rpb4:DSOCR_DN_RPB=4 rpb1:DSOCR_DN_RPB=1 base: rpb4:DSOCR_DN_RPB=4 rpb1:DSOCR_DN_RPB=1 > gpurun_out/rpb_ab.log 2>&1 ;;
    bench8t) run 900 python bench.py --pages-per-gpu 8 --text-pages --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench8t.log 2>&1 ;;
    bench8q) run 900 python bench.py --pages-per-gpu 8 --snapshot q4k --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench8q.log 2>&1 ;;
    rpb_sp) run 600 python tools/ab_trace.py --tokens 256 --rounds 4 --variant base: --variant rpb4:DSOCR_DN_RPB=4 --variant rpb1:DSOCR_DN_RPB=1 --out gpurun_out/rpb_sp.json > gpurun_out/rpb_sp.log 2>&1 ;;
    kvd_sp) run 600 python tools/ab_trace.py --tokens 256 --rounds 3 --variant d150: --variant d0:DSOCR_ATT_KV_DELAY=0 --variant d75:DSOCR_ATT_KV_DELAY=75 --variant d225:DSOCR_ATT_KV_DELAY=225 --variant d300:DSOCR_ATT_KV_DELAY=300 --out gpurun_out/kvd_sp.json > gpurun_out/kvd_sp.log 2>&1 ;;
    split_sp) run 600 python tools/prof_vision.py --reps 5 --variant t512: --variant t0:DSOCR_GEMM_SPLIT_TARGET=0 --variant t256:DSOCR_GEMM_SPLIT_TARGET=256 --variant t1024:DSOCR_GEMM_SPLIT_TARGET=1024 > gpurun_out/split_sp.log 2>&1 ;;
    rb_sp) run 600 python tools/prof_vision.py --reps 5 --variant rb3: --variant rb2:DSOCR_RELBIAS=2 > gpurun_out/rb_sp.log 2>&1 ;;
    rbprof) run 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rbprof -o v --output-format csv -- python tools/prof_vision.py --reps 2 --variant rb3: --variant rb2:DSOCR_RELBIAS=2 > gpurun_out/rbprof.log 2>&1 ;;
    kgrp) run 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm_grouped" > gpurun_out/kgrp.log 2>&1 ;;
    grp_sp) run 600 python tools/prof_vision.py --reps 5 --variant xm1: --variant xm0:DSOCR_GRP_XCD=0 > gpurun_out/grp_sp.log 2>&1 ;;
    scr_sp) run 600 python tools/ab_trace.py --tokens 256 --rounds 4 --variant pre2: --variant pre1:DSOCR_SCREEN_PRE2=0 --out gpurun_out/scr_sp.json > gpurun_out/scr_sp.log 2>&1 ;;
    kscr) run 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -q -m gpu -k "screen" -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/kscr.log 2>&1 ;;
    tatt) run 300 python tools/time_attn_bf16.py --lib new=deepseek-ocr.rs_amd/lib/libdsocr.so --lib old=deepseek-ocr.rs_amd/lib/libdsocr_ab_old.so > gpurun_out/tatt.log 2>&1 ;;
    pmclist) run 60 rocprofv3 -L > gpurun_out/pmclist.txt 2>&1 ;;
    pmcatt1) run 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS -d gpurun_out/pmcatt1 -o pmc --output-format csv -- python3 tools/time_attn_bf16.py --lib ${ATT_LIB:-new=deepseek-ocr.rs_amd/lib/libdsocr.so} --rounds 1 --reps 1 > gpurun_out/pmcatt1.log 2>&1 ;;
    pmcatt2) run 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmcatt2 -o pmc --output-format csv -- python3 tools/time_attn_bf16.py --lib ${ATT_LIB:-new=deepseek-ocr.rs_amd/lib/libdsocr.so} --rounds 1 --reps 1 > gpurun_out/pmcatt2.log 2>&1 ;;
    defer_sp) run 600 python tools/ab_trace.py --tokens 256 --rounds 4 --variant defer: --variant now:DSOCR_ATT_REFILL_DEFER=0 --out gpurun_out/defer_sp.json > gpurun_out/defer_sp.log 2>&1 ;;
    fold_sp) run 600 python tools/ab_trace.py --tokens 256 --rounds 3 --variant fold: --variant nofold:DSOCR_ROUTER_FOLD=0 --out gpurun_out/fold_sp.json > gpurun_out/fold_sp.log 2>&1 ;;
    pmc_l2v) run 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2v -o pmc --output-format csv -- python tools/prof_vision.py --reps 1 > gpurun_out/pmc_l2v.log 2>&1 ;;
    kgemm) run 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm_f32a" > gpurun_out/kgemm.log 2>&1 ;;
    skf_sp) run 600 python tools/prof_vision.py --reps 5 --variant fused: --variant two:DSOCR_SPLITK_FUSED=0 > gpurun_out/skf_sp.log 2>&1 ;;
    adir_sp) run 600 python tools/prof_vision.py --reps 5 --variant adir: --variant lds1:DSOCR_GEMM_ADIR=0 > gpurun_out/adir_sp.log 2>&1 ;;
    gpu_all) run 1100 python -u -m pytest tests -q -m gpu -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 ;;
    smoke) run 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench) run 900 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 ;;
    bench_full) run 1100 python bench.py > gpurun_out/bench_full.log 2>&1 ;;
    prof) DSOCR_NO_GRAPH=1 run 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 ;;
    kbench) run 300 ./tools/kbench $KB_CASES > gpurun_out/kbench.log 2>&1 ;;
    mb) run 120 ./tools/mb_stream > gpurun_out/mb_stream.log 2>&1 ;;
    mbb) run 120 ./tools/mb_barrier > gpurun_out/mb_barrier.log 2>&1 ;;
    mbu) run 120 ./tools/mb_units > gpurun_out/mb_units.log 2>&1 ;;
    pmc_fetch) DSOCR_NO_GRAPH=1 run 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- python bench.py --steps 1 --warmup 0 --max-new-tokens 16 --no-cpu-baseline --roofline-iters 2 > gpurun_out/pmc_fetch.log 2>&1 ;;
    pmc_write) DSOCR_NO_GRAPH=1 run 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc --output-format csv -- python bench.py --steps 1 --warmup 0 --max-new-tokens 16 --no-cpu-baseline --roofline-iters 2 > gpurun_out/pmc_write.log 2>&1 ;;
    pmc_calib) run 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_calib -o mb --output-format csv -- ./tools/mb_stream > gpurun_out/pmc_calib.log 2>&1 ;;
    mbprof) run 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mbprof -o mb --output-format csv -- ./tools/mb_stream > gpurun_out/mbprof.log 2>&1 ;;
    spans1) run 600 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/spans1.log 2>&1 ;;
    spans8) run 600 python bench.py --pages-per-gpu 8 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/spans8.log 2>&1 ;;
    # graph-mode kernel trace with the HIP runtime's graph packet capture off (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0)
    gprof_nopc) DSOCR_SEGV_MAPS=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 run 600 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof_nopc -o g --output-format csv -- python bench.py --steps 1 --warmup 0 --max-new-tokens 64 --no-cpu-baseline --roofline-iters 4 > gpurun_out/gprof_nopc.log 2>&1 ;;
    gprof8_nopc) DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 run 600 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof8_nopc -o g --output-format csv -- python bench.py --pages-per-gpu 8 --steps 1 --warmup 0 --max-new-tokens 64 --no-cpu-baseline --roofline-iters 4 > gpurun_out/gprof8_nopc.log 2>&1 ;;
    # graph-mode trace with packet capture on and the SIGSEGV maps dump armed (the round-2 crash; it no longer
    # reproduces on the round-4 tree: profiles/r04_gprof{32,64}_packet_capture_on.log)
    gprof_maps) DSOCR_SEGV_MAPS=1 run 600 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof_maps -o g --output-format csv -- python bench.py --steps 1 --warmup 0 --max-new-tokens 32 --no-cpu-baseline --roofline-iters 4 > gpurun_out/gprof_maps.log 2>&1 ;;
    k_r4) run 400 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -k "qkv_attention or test_attention or lmhead or screened" -rf -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/k_r4.log 2>&1 ;;
    m_r4) run 600 python -u -m pytest tests/test_gpu_model.py -q -m gpu -k "oproj_route or full_screened" -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/m_r4.log 2>&1 ;;
    dsq_r4) run 900 python -u -m pytest tests/test_dsq.py -q -m gpu -k "full_q4k" -rf -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/dsq_r4.log 2>&1 ;;
    kmoe) run 400 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -k "moe_decode" -rf -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/kmoe${TAG:+_$TAG}.log 2>&1 ;;
    kb_qa) run 180 ./tools/kbench qkvattn1 > gpurun_out/kb_qkvattn.log 2>&1 ;;
    gprof64_maps) DSOCR_SEGV_MAPS=1 run 600 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof64_maps -o g --output-format csv -- python bench.py --steps 1 --warmup 0 --max-new-tokens 64 --no-cpu-baseline --roofline-iters 4 > gpurun_out/gprof64_maps.log 2>&1 ;;
    # graph-mode kernel trace of a whole bench line (512 tokens), default runtime settings
    gprof_full) run 900 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof_full -o g --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/gprof_full.log 2>&1 ;;
    gprof8_full) run 900 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof8_full -o g --output-format csv -- python bench.py --pages-per-gpu 8 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/gprof8_full.log 2>&1 ;;
    gprof128) run 600 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof128 -o g --output-format csv -- python bench.py --steps 1 --warmup 0 --max-new-tokens 128 --no-cpu-baseline > gpurun_out/gprof128.log 2>&1 ;;
    gprof_full_maps) DSOCR_SEGV_MAPS=1 run 900 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof_full_maps -o g --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/gprof_full_maps.log 2>&1 ;;
    kattn) run 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k "attention" > gpurun_out/kattn.log 2>&1 ;;
    katt) run 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k decode_attention > gpurun_out/katt.log 2>&1 ;;
    kb_attn) run 120 ./tools/kbench attn1 attn8 > gpurun_out/kb_attn.log 2>&1 ;;
    # graph-mode kernel trace short enough that the AQL ring never wraps under the profiler
    gprof64) run 600 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof64 -o g --output-format csv -- python bench.py --steps 1 --warmup 0 --max-new-tokens 64 --no-cpu-baseline > gpurun_out/gprof64.log 2>&1 ;;
    gprof64_8) run 600 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof64_8 -o g --output-format csv -- python bench.py --pages-per-gpu 8 --steps 1 --warmup 0 --max-new-tokens 64 --no-cpu-baseline > gpurun_out/gprof64_8.log 2>&1 ;;
    spans8t) run 600 python bench.py --pages-per-gpu 8 --text-pages --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/spans8t.log 2>&1 ;;
    # tagged bench lines (TAG names the log; the caller's environment selects the A/B switches)
    benchx) run 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --roofline-iters 8 > gpurun_out/bench_${TAG:-x}.log 2>&1 ;;
    bench8x) run 600 python bench.py --pages-per-gpu 8 --text-pages --steps 1 --warmup 1 --no-cpu-baseline --roofline-iters 8 > gpurun_out/bench8_${TAG:-x}.log 2>&1 ;;
    benchq4k) run 900 python bench.py --snapshot q4k --pages-per-gpu 8 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/benchq4k.log 2>&1 ;;
    bench8i) run 900 python bench.py --pages-per-gpu 8 --steps 2 --warmup 1 --no-cpu-baseline --roofline-iters 8 > gpurun_out/bench8i${TAG:+_$TAG}.log 2>&1 ;;
    pmc8t_fetch) DSOCR_NO_GRAPH=1 run 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc8t_fetch -o pmc --output-format csv -- python bench.py --pages-per-gpu 8 --text-pages --steps 1 --warmup 0 --max-new-tokens 16 --no-cpu-baseline --roofline-iters 2 > gpurun_out/pmc8t_fetch.log 2>&1 ;;
    pmc8t_write) DSOCR_NO_GRAPH=1 run 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc8t_write -o pmc --output-format csv -- python bench.py --pages-per-gpu 8 --text-pages --steps 1 --warmup 0 --max-new-tokens 16 --no-cpu-baseline --roofline-iters 2 > gpurun_out/pmc8t_write.log 2>&1 ;;
    gprof8t_nopc) DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 run 600 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof8t_nopc -o g --output-format csv -- python bench.py --pages-per-gpu 8 --text-pages --steps 1 --warmup 0 --max-new-tokens 64 --no-cpu-baseline --roofline-iters 4 > gpurun_out/gprof8t_nopc.log 2>&1 ;;
    pmcdots_fetch) run 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcdots_fetch -o pmc --output-format csv -- python bench.py --workload dots2048 --steps 1 --warmup 0 > gpurun_out/pmcdots_fetch.log 2>&1 ;;
    # MFMA busy per kernel over one dots page (tools/pmc_mfma.py reads the csv)
    pmc_mfma_dots) run 900 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_mfma_dots -o pmc --output-format csv -- python bench.py --workload dots2048 --steps 1 --warmup 0 > gpurun_out/pmc_mfma_dots.log 2>&1 ;;
    pmcdots_write) run 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcdots_write -o pmc --output-format csv -- python bench.py --workload dots2048 --steps 1 --warmup 0 > gpurun_out/pmcdots_write.log 2>&1 ;;
    # round 5
    counters) run 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 ;;
    # MFMA utilisation of the vision / prefill kernels (eager launches; decode shortened to 8 tokens)
    pmc_mfma) grep -q SQ_VALU_MFMA_BUSY_CYCLES gpurun_out/counters.txt && DSOCR_NO_GRAPH=1 run 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_mfma -o pmc --output-format csv -- python bench.py --steps 1 --warmup 0 --max-new-tokens 8 --trace-only ${PMC_ARGS} > gpurun_out/pmc_mfma${TAG:+_$TAG}.log 2>&1 ;;
    # production-only graph-mode kernel trace of the whole bench line (512 tokens): packet capture on (the
    # runtime default), an AQL ring of 131072 packets so the profiler's ring-wrap read never happens
    gprod) ROC_AQL_QUEUE_SIZE=131072 run 900 rocprofv3 --kernel-trace --stats -d gpurun_out/gprod${TAG:+_$TAG} -o g --output-format csv -- python bench.py --steps 1 --warmup 0 --trace-only ${BENCH_ARGS} > gpurun_out/gprod${TAG:+_$TAG}.log 2>&1 ;;
    benchr) run 900 python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/benchr${TAG:+_$TAG}.log 2>&1 ;;
    kb_moe1) KB_WAVES=1 run 180 ./tools/kbench moe1 > gpurun_out/kb_moe1_o0.log 2>&1 && DSOCR_GU_ORDER=1 KB_WAVES=1 run 180 ./tools/kbench moe1 > gpurun_out/kb_moe1_o1.log 2>&1 ;;
    # same-process A/B under a graph-mode kernel trace (AB_VARIANTS: the --variant arguments)
    ab) ROC_AQL_QUEUE_SIZE=131072 run 900 rocprofv3 --kernel-trace --stats -d gpurun_out/ab${TAG:+_$TAG} -o g --output-format csv -- python tools/ab_trace.py --out gpurun_out/ab${TAG:+_$TAG}/order.json ${AB_ARGS} > gpurun_out/ab${TAG:+_$TAG}.log 2>&1 ;;
    # PMC traffic with every MoE launch priced at its own routing (tools/pmc_decode.py + pmc_summary.py --routing);
    # PMC_RUN = b1 | b8 | b8i
    pmcr) case ${PMC_RUN:-b1} in b1) A="--pages 1" ;; b8) A="--pages 8 --text-pages" ;; b8i) A="--pages 8" ;; esac
          for C in FETCH_SIZE WRITE_SIZE; do DSOCR_NO_GRAPH=1 run 600 rocprofv3 --pmc $C -d gpurun_out/pmc_${PMC_RUN:-b1}_$C -o pmc --output-format csv -- python tools/pmc_decode.py $A --tokens 16 --out gpurun_out/routing_${PMC_RUN:-b1}.json > gpurun_out/pmc_${PMC_RUN:-b1}_$C.log 2>&1 || exit 1; done ;;
    envab) run 900 tools/env_ab.sh ${ENV_AB} > gpurun_out/envab${TAG:+_$TAG}.log 2>&1 ;;
    kb_router8) run 180 ./tools/kbench router8 > gpurun_out/kb_router8${TAG:+_$TAG}.log 2>&1 ;;
    parity8) DSOCR_PARITY_OUT=gpurun_out/parity8${TAG:+_$TAG}.jsonl run 900 python -u -m pytest tests/test_full_parity.py -q -m gpu -rf -p no:cacheprovider --timeout 400 --timeout-method thread -k "batch8" > gpurun_out/parity8${TAG:+_$TAG}.log 2>&1 ;;
    *) echo "unknown step $step" >> gpurun_out/rc.log ;;
  esac
done
