#!/usr/bin/env python3
"""DeepSeek-OCR page throughput on MI355X (BASELINE.json metric).

A *step* = one pass of the page path over one batch of synthetic input: for every
page of the batch, vision tower (SAM + CLIP + projector) -> 706-token prefill ->
512 greedy decode tokens (EOS ignored, no_repeat_ngram_size = 20), exactly the
reference's OcrEngine::decode work per page.  Default workload =
BASELINE configs[1]: one 1024x1024 page per GPU per step (DeepSeek-OCR, weights
fp16-rounded as the reference's `--dtype f16`, f32 compute).  `--pages-per-gpu 8`
with 8 GPUs is configs[2] (batch 64, data parallel).

Multi-GPU: one process per GPU (torchrun), pages sharded by index, no data-path
collective; a CPU gloo group only provides the barrier and the max-over-ranks time.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "deepseek-ocr.rs_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def blas_threads():
    """Threads the oracle's BLAS actually runs with (numpy's OpenBLAS pool)."""
    try:
        from threadpoolctl import threadpool_info
        n = [p["num_threads"] for p in threadpool_info() if p.get("user_api") == "blas"]
        if n:
            return int(max(n))
    except Exception:
        pass
    return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))


def visible_gpus():
    import ctypes as C

    from dsocr._lib import lib
    n = C.c_int(0)
    return n.value if lib().dsocr_device_count(C.byref(n)) == 0 else 1


def relaunch_under_torchrun(n):
    """`bench.py --gpus N` with no launcher: run N ranks under torch.distributed.run as a CHILD process
    (this process has made no HIP call yet) and return its exit code.  The ranks see WORLD_SIZE and
    take the normal path below."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] --gpus {n} without a launcher: {' '.join(cmd)}")
    return subprocess.run(cmd).returncode


def rank_devices(dist, local):
    """Device ordinal of every rank (rank order)."""
    if dist is None:
        return [local]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, local)
    return out


def page_indices(step, world, rank, ppg):
    """Pages of one bench step on one rank: rank r of W takes pages [(step*W + r)*ppg, +ppg) —
    disjoint across ranks and steps (data parallel, no collective on the data path)."""
    base = (step * world + rank) * ppg
    return list(range(base, base + ppg))


def reduce_over_ranks(dist, elapsed, tok_s):
    """Job time = max over ranks (the slowest rank ends the step); decode tok/s = sum."""
    if dist is None:
        return elapsed, tok_s
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    r = torch.tensor([tok_s], dtype=torch.float64)
    dist.all_reduce(r, op=dist.ReduceOp.SUM)
    return float(t.item()), float(r.item())


def pmc_traffic(kernel_prefix, runs=None):
    """HBM bytes per launch of a kernel from the committed rocprofv3 PMC summary (latest
    profiles/rNN_pmc_traffic.json, tools/pmc_summary.py + tools/pmc_merge.py: FETCH_SIZE x 2 (gfx950 reports half of
    wide streaming reads) + WRITE_SIZE, each from its own --pmc pass) -> (bytes, traffic / algorithmic or None).
    `runs` names the PMC runs whose workload matches this bench line (b1: one page; b8: 8 text pages; b8i: 8 image
    pages).  Round 5: the MoE launches of a run are priced one by one at their own distinct experts
    (tools/pmc_decode.py), so bytes and ratio come from the same launches; a kernel measured only in another run
    gives (None, None)."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")))
    try:
        d = json.load(open(paths[-1]))
    except Exception:
        return None, None
    for table in ("kernels", "kernels_b8", "kernels_b8i", "kernels_dots"):
        for name, v in d.get(table, {}).items():
            if name.startswith(kernel_prefix) and (runs is None or v.get("run") in runs):
                if v.get("priced_hbm_bytes_per_launch"):
                    return v["priced_hbm_bytes_per_launch"], v.get("traffic_over_algorithmic")
                return v.get("hbm_bytes_per_launch"), None
    return None, None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


CORES_ALL_STEPS = 16       # decode forwards timed by the all-CPU leg (scaled to the page's max_new - 1)
CORES_ALL_DEADLINE_S = 150  # the all-CPU leg's child process is stopped after this


def cpu_quota():
    """CPUs the job's cgroup may use (cpu.max quota / period), or None when unlimited / unreadable."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_leg(threads, page, tok_ids, mask, max_new, steps):
    """One page of the workload on `threads` OpenMP threads of the C++ restatement (oracle/cpu_ref.cpp): the
    vision tower (cv_features), then the 706-token prefill and (steps - 1) decode forwards (cr_generate with the
    greedy 20-gram ban), the decode time scaled to the page's (max_new - 1) forwards when steps < max_new."""
    import numpy as np

    import dsocr
    from oracle import cpu_ref
    from oracle.weights import Weights
    cfg = json.load(open(dsocr.FULL_CONFIG))
    cpu_ref.set_threads(threads)
    t = time.time()
    cv = cpu_ref.CpuVision(cfg, Weights(seed=0, dtype="f16"), threads=threads)
    log(f"[cpu] {threads} threads: C++ vision tower loaded in {time.time() - t:.1f}s")
    t0 = time.time()
    emb, _ = cv.embeddings(page)
    vision_s, vis_ms = time.time() - t0, dict(cv.last_ms)
    del cv
    log(f"[cpu] {threads} threads: vision {vision_s:.2f}s")
    t = time.time()
    cr = cpu_ref.CpuRef(cfg, Weights(seed=0, dtype="f16"), threads=threads)
    log(f"[cpu] {threads} threads: C++ decoder loaded in {time.time() - t:.1f}s, decoding {steps - 1} steps")
    ids, ms = cr.generate(np.asarray(tok_ids, np.int64), np.asarray(mask, np.uint8), emb, steps, ngram=20)
    cr.close()
    prefill_s, decode_s = ms["prefill_ms"] / 1e3, ms["decode_ms"] / 1e3 * (max_new - 1) / max(1, steps - 1)
    page_s = vision_s + prefill_s + decode_s
    scaled = "" if steps == max_new else f", scaled from {steps - 1} timed steps"
    log(f"[cpu] {threads} threads: vision {vision_s:.2f}s prefill {prefill_s:.2f}s decode {decode_s:.2f}s{scaled}")
    return {"value": 1.0 / page_s, "unit": "pages/s", "cores": threads,
            "decode_tok_s": (max_new - 1) / decode_s,
            "stage_s": {"vision": round(vision_s, 3), "prefill": round(prefill_s, 3), "decode": round(decode_s, 3)},
            "vision_ms": {k: round(v, 1) for k, v in vis_ms.items()},
            "sample": f"1 synthetic 1024x1024 page: vision {vision_s:.2f}s (C++, incl. numpy preprocessing) + "
                      f"prefill {prefill_s:.2f}s ({len(tok_ids)} tok, C++) + {max_new - 1} decode steps "
                      f"{decode_s:.2f}s (C++, {decode_s / max(1, max_new - 1) * 1e3:.1f} ms/step{scaled}), "
                      f"{threads} threads; first ids {[int(i) for i in ids[:4]]}"}


def cpu_leg_child(d):
    """`bench.py --cpu-leg DIR`: the all-CPU leg in its own process (no GPU: nothing here touches HIP), inputs
    from DIR/leg.npz, the run record to DIR/leg.json."""
    import numpy as np
    z = np.load(os.path.join(d, "leg.npz"))
    run = cpu_leg(int(z["threads"]), z["page"], z["tok_ids"], z["mask"], int(z["max_new"]), int(z["steps"]))
    json.dump(run, open(os.path.join(d, "leg.json"), "w"))


def cpu_baseline(pages, tok_ids, mask, max_new, decode_steps=0):
    """The repo's C++ / OpenMP CPU restatement of the page path (oracle/cpu_ref.cpp, test/bench infrastructure)
    timed on rank 0's host cores, one whole page of the workload: the vision tower (cv_features: SAM-ViTDet-B +
    CLIP-L + projector, packed-panel AVX-512 GEMMs, the oracle's numpy preprocessing and token formatting), then
    the decoder (cr_generate: the 706-token prefill and ALL (max_new - 1) decode forwards with the greedy
    20-gram-ban selection), timed whole (no extrapolation).  Threads: OMP_NUM_THREADS (the job's CPU share: 16 on
    the GPU box).  Stage sums are reported like the reference's bench (crates/cli/src/bench.rs:200-260: vision,
    prefill, decode); the vision embeddings are checked against the numpy oracle's in tests/test_cpu_ref.py.
    `cores_all`: the same page on every CPU the process may run on (allowed_cpus), in a child process with
    OMP_WAIT_POLICY=passive (256 spinning threads against a 16-CPU cgroup quota stall on every barrier), its
    decode a bounded sample of CORES_ALL_STEPS forwards, stopped after CORES_ALL_DEADLINE_S."""
    import subprocess
    import tempfile

    import numpy as np
    allowed = len(os.sched_getaffinity(0))
    threads = int(os.environ.get("OMP_NUM_THREADS") or allowed)
    out = cpu_leg(threads, pages[0], tok_ids, mask, max_new, max_new)
    out.update({"kind": "cpp",
                "port": "oracle/cpu_ref.cpp: C++ / OpenMP restatement of the whole page path (vision tower + decoder, "
                        "AVX-512 micro-kernels, f32 math); the Rust reference cannot be built here",
                "host_cpus": os.cpu_count(), "allowed_cpus": allowed, "cpu_quota_cpus": cpu_quota(),
                "cpu_model": cpu_model(),
                "threads_note": "value: the job's CPU share (OMP_NUM_THREADS); cores_all: every allowed CPU"})
    if allowed == threads or os.environ.get("DSOCR_CPU_ONE_COUNT"):
        return out
    with tempfile.TemporaryDirectory() as d:
        np.savez(os.path.join(d, "leg.npz"), page=np.asarray(pages[0]), tok_ids=np.asarray(tok_ids, np.int64),
                 mask=np.asarray(mask, np.uint8), threads=allowed, max_new=max_new,
                 steps=min(max_new, CORES_ALL_STEPS + 1))
        env = dict(os.environ, OMP_NUM_THREADS=str(allowed), OMP_WAIT_POLICY="passive")
        log(f"[cpu] {allowed} threads: child process (deadline {CORES_ALL_DEADLINE_S} s)")
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-leg", d], env=env, cwd=ROOT)
        t0 = time.time()
        while p.poll() is None and time.time() - t0 < CORES_ALL_DEADLINE_S:
            time.sleep(1)
        if p.poll() is None:
            p.kill()
            p.wait()
            log(f"[cpu] {allowed} threads: stopped at the {CORES_ALL_DEADLINE_S} s deadline")
            out["cores_all"] = {"cores": allowed, "value": None, "status": f"not finished in {CORES_ALL_DEADLINE_S} s "
                                f"(cgroup quota {cpu_quota()} CPUs)"}
        elif p.returncode == 0:
            out["cores_all"] = json.load(open(os.path.join(d, "leg.json")))
        else:
            out["cores_all"] = {"cores": allowed, "value": None, "status": f"child exited {p.returncode}"}
    return out


SPAN_HZ = 100e6  # s_memrealtime


def lang_dims(cfg):
    """Decoder dimensions the span pricing needs (the checkpoint's language_config)."""
    c = cfg.get("language_config", cfg)
    heads, kvh = c["num_attention_heads"], c["num_key_value_heads"]
    H = c["hidden_size"]
    hd = H // heads
    return {"H": H, "I": c["moe_intermediate_size"], "Is": c["moe_intermediate_size"] * c.get("n_shared_experts", 0),
            "K": c["num_experts_per_tok"], "heads": heads, "kv_heads": kvh, "hd": hd, "qkvn": (heads + 2 * kvh) * hd}


def span_bytes(kind, d, B, P, experts, step):
    """Algorithmic HBM bytes of one decode launch: 16-bit weights streamed once + f32 activations.
    gate/up: the distinct routed experts' gate+up rows + the shared expert's, x in, h out; down: their
    down rows, h in, residual read + write; attention: f32 K and V of every attended key (page b at
    step s attends P + s keys) + the q/k/v row in and the context row out."""
    H, I, Is, K = d["H"], d["I"], d["Is"], d["K"]
    if kind == "moe_gateup":
        return (experts * 2 * I + 2 * Is) * H * 2 + B * H * 4 + (B * K * I + B * Is) * 4
    if kind == "moe_down":
        return (experts * I + Is) * H * 2 + (B * K * I + B * Is) * 4 + 2 * B * H * 4
    return B * (P + step) * d["kv_heads"] * d["hd"] * 4 * 2 + B * (d["qkvn"] + H) * 4


def span_roofline(spans, d, B, P):
    """Per kind, over every decode launch of the generate (each priced from its own expert count / step):
    launches; `avg_us` = mean dispatch duration (HIP events recorded around the launch inside the replayed
    step graph, what rocprofv3's kernel trace reports; the in-kernel wave span when no events were taken)
    and `GB/s` = sum of algorithmic bytes / sum of those durations; `wave_avg_us` / `wave_GB/s` the same
    over the in-kernel span (first wave entry -> last wave exit, s_memrealtime) where recorded."""
    import numpy as np
    out = {}
    for kind, arr in spans.items():
        valid = (arr[..., 4] > 0) | (arr[..., 0] > 0)
        layer, step = np.nonzero(valid)
        if not len(layer):
            continue
        rec = arr[layer, step]
        ev = rec[:, 4].astype(np.float64) * 1e-9
        has_wave = rec[:, 0] > 0
        wave = (rec[:, 1].astype(np.int64) - rec[:, 0].astype(np.int64)) / SPAN_HZ
        events = bool(np.all(ev > 0))
        dur = ev if events else wave
        ex = rec[:, 2].astype(np.int64)
        by = np.array([span_bytes(kind, d, B, P, int(e), int(s)) for e, s in zip(ex, step)], np.float64)
        o = {"launches": int(len(dur)), "avg_us": float(dur.mean() * 1e6),
             "p50_us": float(np.median(dur) * 1e6), "max_us": float(dur.max() * 1e6),
             "bytes_per_launch": float(by.mean()), "GB/s": float(by.sum() / dur.sum() / 1e9),
             "frac": float(by.sum() / dur.sum() / 1e9 / HBM_PEAK_GBS),
             "timing": "hip events in graph" if events else "in-kernel wave span",
             "experts_mean": float(ex.mean()), "experts_range": [int(ex.min()), int(ex.max())]}
        if np.all(has_wave):
            o["wave_avg_us"] = float(wave.mean() * 1e6)
            o["wave_GB/s"] = float(by.sum() / wave.sum() / 1e9)
        out[kind] = o
    return out


def dots_flops(cfg, N):
    """Algorithmic FLOPs of the dots.ocr vision tower on N patch tokens (one frame): per block the
    qkv / proj / fc1 / fc3 / fc2 GEMMs 2 N D (3D + D + 3 I) and the attention 4 N^2 D (QK^T and P.V);
    patch embed 2 N (3 p^2) D; merger 2 (N/4) (G^2 + G H)."""
    D, I, L = cfg["embed_dim"], cfg["intermediate_size"], cfg["num_hidden_layers"]
    G = D * cfg["spatial_merge_size"] ** 2
    gemm_block = 2.0 * N * D * (3 * D + D + 3 * I)
    attn_block = 4.0 * N * N * D
    other = 2.0 * N * 3 * cfg["patch_size"] ** 2 * D + 2.0 * (N / 4) * (G * G + G * cfg["hidden_size"])
    return gemm_block * L, attn_block * L, other


def run_dots(args, rank, world, local, dist):
    """BASELINE configs[3]: dots.ocr (bf16) vision tower on a 2048 x 2048 page per GPU per step (the
    reference's smart_resize maps it to 2044 x 2044, fast_image_resize's Catmull-Rom pass resizes it,
    grid 146 x 146 = 21316 patch tokens; preprocessing on the host before the timed region)."""
    import ctypes as C

    import numpy as np

    from dsocr._lib import check, lib
    from dsocr.dots import DOTS_CONFIG, DotsVision, preprocess
    from dsocr.synth import synthetic_page
    L = lib()
    t_load = time.time()
    eng = DotsVision(DOTS_CONFIG, synthetic_seed=0, device=local)
    log(f"[rank {rank}] dots vision tower loaded on hip:{local} in {time.time() - t_load:.1f}s")
    cfg = json.load(open(DOTS_CONFIG))["vision_config"]
    size = args.dots_size
    ppg = args.pages_per_gpu

    def dev(arr):
        p = C.c_void_p()
        check(L.dsocr_dev_alloc(arr.nbytes, C.byref(p)))
        check(L.dsocr_memcpy_h2d(p, arr.ctypes.data_as(C.c_void_p), arr.nbytes))
        return p

    pages = []  # inputs resident in HBM before the timed region
    for s in range(args.warmup + args.steps):
        batch = []
        for idx in page_indices(s, world, rank, ppg):
            patches, grid = preprocess(DOTS_CONFIG, synthetic_page(idx, size, size))
            batch.append((dev(patches), grid))
        pages.append(batch)
    N = grid[0] * grid[1] * grid[2]
    groups = N // 4
    out = C.c_void_p()
    check(L.dsocr_dev_alloc(groups * eng.hidden * 4, C.byref(out)))
    for s in range(args.warmup):
        for p, g in pages[s]:
            eng.embed_device(p, g, out)
    check(L.dsocr_dev_sync())
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for s in range(args.warmup, args.warmup + args.steps):
        for p, g in pages[s]:
            eng.embed_device(p, g, out)
    check(L.dsocr_dev_sync())
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed, _ = reduce_over_ranks(dist, elapsed, 0.0)
    value = args.steps * ppg * world / elapsed
    if rank != 0:
        return None
    # one more page with its first 4 layers' attention timed alone (events around each launch)
    eng.embed_device(pages[-1][0][0], pages[-1][0][1], out, time_attention_layers=4)
    tm = eng.last_timings()
    gemm_f, attn_f, other_f = dots_flops(cfg, N)
    attn_layer_ms = tm["attention_ms"] / 4
    attn_tf = (attn_f / cfg["num_hidden_layers"]) / (attn_layer_ms * 1e-3) / 1e12
    planes = 2 if os.environ.get("DSOCR_DOTS_PV_PLANES") == "2" else 3
    issue = (1 + planes) / 2.0
    page_ms = elapsed / (args.steps * ppg) * 1e3
    return {
        "metric": "pages/sec, dots.ocr bf16 vision tower, 2048px page (BASELINE configs[3])",
        "value": round(value, 4), "unit": "pages/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("bf16 (reference semantics: bf16 tensors between ops; f32 attention math, P.V with f32 P: "
                  "exact 3-plane)" if planes == 3 else
                  "bf16 (bf16 tensors between ops; f32 scores/softmax; P.V on 2 bf16 planes of P, 16 significant "
                  "bits: DSOCR_DOTS_PV_PLANES=2, narrower than the reference)"),
        "data": "synthetic document pages + seeded synthetic weights (no checkpoint offline)",
        "config": {"workload": f"configs[3]: dots.ocr vision tower, {size}x{size} page (resized to "
                               f"{grid[1] * 14}x{grid[2] * 14}), grid {grid[1]}x{grid[2]}, "
                               f"{N} patch tokens, {groups} output rows", "pages_per_gpu": ppg,
                   "global_batch": ppg * world, "parallelism": f"dp{world}"},
        "stage_ms": {"page_ms": round(page_ms, 2), "blocks_ms": round(tm["blocks_ms"], 2),
                     "patch_ms": round(tm["patch_ms"], 2), "merger_ms": round(tm["merger_ms"], 2)},
        # achieved = the reference's attention FLOPs (QK^T + P.V, f32 math) / the kernel's time; the kernel
        # runs them on the bf16 matrix cores (1 exact pass for QK^T; P.V on 3 bf16 planes of P — exact, the
        # reference's f32 P; DSOCR_DOTS_PV_PLANES=2 opts into 16 significant bits), so the peak is the dense bf16 MFMA rate and the issued
        # MFMA work is (1 + planes) / 2 x the algorithmic FLOPs
        "roofline": {"bound": "mfma", "achieved": round(attn_tf, 2), "peak": 2500.0, "unit": "TFLOP/s",
                     "frac": round(attn_tf / 2500.0, 4), "traffic": pmc_traffic("attention_bf16_tr_kernel")[0],
                     "mfma_issued_tflops": round(issue * attn_tf, 2), "mfma_issued_frac": round(issue * attn_tf / 2500.0, 4),
                     "kernel": f"attention_bf16_tr_kernel<128, {planes}> (bidirectional flash attention over the page's "
                               f"21316 tokens on v_mfma_f32_32x32x16_bf16 with the reference's f32 math: exact bf16 q.k "
                               f"products, P split into {planes} bf16 planes for P.V)",
                     "avg_launch_us": round(attn_layer_ms * 1e3, 1),
                     "flops_per_launch": attn_f / cfg["num_hidden_layers"],
                     "tower_tflops_total": round((gemm_f + attn_f + other_f) / 1e12, 2),
                     "tower_achieved_tflops": round((gemm_f + attn_f + other_f) / (page_ms * 1e-3) / 1e12, 2)},
        "cpu_baseline": None,
    }


def chain_roofline(chain, waves, d, B, P):
    """Dispatch-level durations from a chain-span generate (dsocr_engine_set_spans 4): every layer's attention,
    o_proj, router, gate/up and down launches stamp their waves (one fold per step, nothing between launches),
    so duration = last wave exit of the launch - last wave exit of the launch before it (its boundary
    included, as a back-to-back rocprofv3 dispatch record), boundary = its first wave entry - that exit.
    MoE launches are priced at the distinct experts the wave-span generate of the same batch recorded."""
    import numpy as np
    # the launch before each kind (layer offset); at 3..8 pages the gate/up launch routes itself (no router launch):
    # its predecessor is then the o_proj launch
    pred = {"moe_gateup": (("router", 0), ("o_proj", 0)), "moe_down": (("moe_gateup", 0),),
            "o_proj": (("attention", 0),), "router": (("o_proj", 0),), "attention": (("moe_down", -1),)}
    Hh, hd, heads = d["H"], d["hd"], d["heads"]
    out = {}
    for kind, cands in pred.items():
        a = chain.get(kind)
        cands = [(chain[pk], dl) for pk, dl in cands if pk in chain and np.any(chain[pk][..., 1] > 0)]
        if a is None or not cands or (kind == "attention" and B > 1):  # (B > 1: an unstamped q/k/v launch precedes it)
            continue
        b, dl = cands[0]
        L, S = a.shape[0], a.shape[1]
        durs, bnds, wv, by = [], [], [], []
        for l in range(max(0, -dl), L):
            for st in range(S):
                e_in, e_out, p_out = int(a[l, st, 0]), int(a[l, st, 1]), int(b[l + dl, st, 1])
                if not (e_in and e_out and p_out) or e_out <= p_out:
                    continue
                durs.append((e_out - p_out) / SPAN_HZ)
                bnds.append((e_in - p_out) / SPAN_HZ)
                wv.append((e_out - e_in) / SPAN_HZ)
                if kind in ("moe_gateup", "moe_down"):
                    ex = int(waves[kind][l, st, 2]) if kind in waves else d["K"] * B
                    by.append(span_bytes(kind, d, B, P, ex, st))
                elif kind == "attention":
                    by.append(span_bytes(kind, d, B, P, 0, st) + 3 * Hh * Hh * 2)  # + the fused q/k/v weights (B = 1)
                elif kind == "o_proj":
                    by.append(heads * hd * Hh * 2 + B * (heads * hd + 2 * Hh) * 4)
                else:
                    by.append(64 * Hh * 2 + B * Hh * 4)
        if not durs:
            continue
        du = np.array(durs)
        bb = np.array(by, np.float64)
        out[kind] = {"launches": len(durs), "avg_us": float(du.mean() * 1e6), "p50_us": float(np.median(du) * 1e6),
                     "boundary_us": float(np.mean(bnds) * 1e6), "wave_us": float(np.mean(wv) * 1e6),
                     "bytes_per_launch": float(bb.mean()), "GB/s": float(bb.sum() / du.sum() / 1e9),
                     "frac": float(bb.sum() / du.sum() / 1e9 / HBM_PEAK_GBS)}
    return out


def persist_bytes(cfg, L_keys):
    """Algorithmic HBM bytes of one persistent decode launch (every decoder layer of one step, one page): each
    layer's f16 weights once (q/k/v, o_proj, router, the 6 picked experts' gate/up/down, the shared experts; the
    dense layer's MLP), its f32 K and V over the L_keys - 1 cached keys read + the new key written, the norm
    weights; hand-off granules are not algorithmic."""
    c = cfg.get("language_config", cfg)
    H, heads = c["hidden_size"], c["num_attention_heads"]
    hd = H // heads
    I, E_k, n_sh = c["moe_intermediate_size"], c["num_experts_per_tok"], c.get("n_shared_experts", 0)
    Is, Id, nl = I * n_sh, c["intermediate_size"], c["num_hidden_layers"]
    dense = c.get("first_k_dense_replace", 0)
    attn = 3 * heads * hd * H * 2 + H * heads * hd * 2 + 2 * H * 4
    moe = c["n_routed_experts"] * H * 2 + 3 * (E_k * I + Is) * H * 2
    mlp_dense = 3 * Id * H * 2
    kv = heads * hd * 4 * 2 * (L_keys - 1) + heads * hd * 4 * 2
    return nl * (attn + kv) + dense * mlp_dense + (nl - dense) * moe, (E_k * I) * H * 2 * 3


def persist_roofline(eng, batch, params, ppg, args):
    """Roofline of the one-page decode as it runs: ONE persistent launch per step (decode_persist.hip) holds every
    decoder layer, so it is the dominant kernel.  A generate of the first timed batch with HIP events around each
    persistent launch (the dispatch-level duration rocprofv3 reports for dec_persist_kernel) and the kernel's
    phase clocks: achieved = algorithmic bytes of each launch (persist_bytes at its step's key count) summed over
    the generate / the summed launch durations.  `moe_routed`: the routed experts' gate + up + down bytes (6 x 3 x
    896 x 1280 f16 per layer) over the routed phase of each layer (picks known on the first workgroup -> the last
    workgroup's split-K partial stored), the window that holds every routed expert byte (the shared expert's rows
    stream earlier, beside the attention hand-offs)."""
    import numpy as np
    import dsocr
    cfg = json.load(open(dsocr.FULL_CONFIG))
    nl = cfg.get("language_config", cfg)["num_hidden_layers"]
    P = len(batch[0][0])
    eng.set_persist_stamps(1)
    eng.generate_batch(batch, params, ignore_eos=True)
    info = eng.persist_info(layers=nl)
    us = np.asarray(info["launch_us"], np.float64)
    st = info["stamps"][: len(us)].astype(np.int64)  # [steps][256][layers][9]
    n = len(us)
    byts = np.array([persist_bytes(cfg, P + i + 1)[0] for i in range(n)], np.float64)
    routed_b = persist_bytes(cfg, P)[1]
    gbs = byts.sum() / (us.sum() * 1e-6) / 1e9
    # phase windows over the workgroups (s_memrealtime, 100 MHz), per step and layer
    first = st.min(axis=1)  # [steps][layers][9]
    last = st.max(axis=1)
    dense = cfg.get("language_config", cfg).get("first_k_dense_replace", 0)
    routed_s = (last[:, dense:, 7] - first[:, dense:, 6]) / SPAN_HZ
    layer_s = (last[:, :, 8] - first[:, :, 0]) / SPAN_HZ
    phase_names = ("x gathered", "q/k/v published", "attention partials", "merge -> ctx published",
                   "ctx gathered", "x_new normalised + picks", "split-K partials", "x_{l+1} published")
    # per phase: mean over steps and layers of (last workgroup at phase k) - (last workgroup at phase k - 1)
    ph = {phase_names[k - 1]: round(float(np.mean(last[:, :, k] - last[:, :, k - 1]) / SPAN_HZ * 1e6), 2)
          for k in range(1, 9)}
    rt_gbs = routed_b * routed_s.size / routed_s.sum() / 1e9
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": pmc_traffic("dec_persist_kernel", runs=("b1",))[0],
            "kernel": "dec_persist_kernel (one decode step: all decoder layers of the page in ONE persistent launch)",
            "avg_launch_us": round(float(us.mean()), 2), "p50_launch_us": round(float(np.median(us)), 2),
            "launches": int(n), "bytes_per_launch": round(float(byts.mean())),
            "timing": "HIP events around every persistent launch inside the replayed step graph",
            "layer_us": round(float(layer_s.mean() * 1e6), 2),
            "phase_us": ph,
            "moe_routed": {"bytes_per_layer": routed_b, "window_us": round(float(routed_s.mean() * 1e6), 2),
                           "GB/s": round(rt_gbs, 1), "frac": round(rt_gbs / HBM_PEAK_GBS, 4),
                           "window": "picks known (first workgroup) -> split-K partials stored (last workgroup)"},
            "kv_len": [P + 1, P + n]}


def decode_roofline(eng, batch, params, ppg, args):
    """The roofline object of the decode MoE gate/up (the north-star kernel) at this batch size (rank 0, after the
    timed region, on the first timed batch):
      1. profile_decode: one decode step's layers replayed as a graph with and without the gate/up launches, HIP
         events around the replays -> `avg_launch_us`, `achieved`, `frac` (the launch's in-context dispatch cost;
         the round-5 production rocprofv3 trace agrees with it, profiles/INDEX_r05.md);
      2. chain spans over a whole generate (every layer's attention, o_proj, router, gate/up, down launches stamp
         their waves; one fold per step, nothing between the launches): exit-to-exit durations with the boundary
         before each launch -> `chain`;
      3. in-kernel wave spans with each MoE launch's distinct experts (one fold launch after each stamped launch)
         -> `in_kernel_waves` and the pricing of (2) (same batch, same routing: ids checked equal)."""
    import dsocr
    dims = lang_dims(json.load(open(dsocr.FULL_CONFIG)))
    P = len(batch[0][0])
    eng.set_spans(eng.SPAN_WAVES)
    ids_w = eng.generate_batch(batch, params, ignore_eos=True)
    spans_w = eng.spans()
    eng.set_spans(eng.SPAN_CHAIN)
    ids_c = eng.generate_batch(batch, params, ignore_eos=True)
    spans_c = eng.spans()
    eng.set_spans(0)
    if ids_w != ids_c:
        raise RuntimeError("span generates of one batch emitted different ids")
    waves = span_roofline(spans_w, dims, ppg, P)
    chain = chain_roofline(spans_c, spans_w, dims, ppg, P)
    prof = eng.profile_decode(args.roofline_iters)
    kernel = prof["moe_gateup_kernel"]  # what the dispatch runs at this batch size

    def ctx_line(k):
        p = prof[k]
        return {"ctx_us": round(p["ctx_us"], 3), "bytes": p["bytes"],
                "GB/s": round(p["bytes"] / (p["ctx_us"] * 1e-6) / 1e9, 1) if p["ctx_us"] > 0 else None,
                "frac": round(p["bytes"] / (p["ctx_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) if p["ctx_us"] > 0 else None,
                "isolated_us": round(p["avg_us"], 3), "replay_us": round(p["replay_us"], 3)}
    gu = ctx_line("moe_gateup")
    dn = ctx_line("moe_down")
    # the whole MoE of a layer as SURVEY 8(d) prices it: gate + up + down bytes over both launches' durations
    tot_b, tot_us = gu["bytes"] + dn["bytes"], gu["ctx_us"] + dn["ctx_us"]
    moe_total = {"bytes_per_layer": tot_b, "ctx_us": round(tot_us, 3),
                 "GB/s": round(tot_b / (tot_us * 1e-6) / 1e9, 1) if tot_us > 0 else None,
                 "frac": round(tot_b / (tot_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) if tot_us > 0 else None}
    if chain.get("moe_gateup") and chain.get("moe_down"):
        cu = chain["moe_gateup"]["avg_us"] + chain["moe_down"]["avg_us"]
        moe_total.update({"chain_us": round(cu, 3), "chain_frac": round(tot_b / (cu * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)})
    runs = ("b1",) if ppg == 1 else (("b8",) if args.text_pages and ppg == 8 else (("b8i",) if ppg == 8 else ()))
    traffic, ratio = pmc_traffic(kernel, runs=runs)
    return {"bound": "hbm", "achieved": gu["GB/s"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": gu["frac"], "traffic": traffic, "traffic_over_algorithmic": ratio,
            "kernel": kernel + " (decode MoE gate/up of one layer: routed top-6 experts per page + shared experts)",
            # avg_launch_us = the launch's dispatch-level cost in the production chain, by HIP events on the engine
            # stream: one decode step's layers captured as a graph twice (as the decode loop runs them, and without
            # the gate/up launches), each replayed back to back between events; (full - without) / MoE layers.
            # Round 5: the 512-token graph-mode rocprofv3 trace of the timed generate alone (packet capture on, AQL
            # ring 131072) gives the same figure for the same tree (profiles/INDEX_r05.md); bytes priced at the
            # routing the replayed step takes (experts_touched distinct experts)
            "avg_launch_us": gu["ctx_us"], "bytes_per_launch": gu["bytes"],
            "experts_touched": prof["experts_touched"],
            "timing": "HIP events: step-graph replays with and without the gate/up launches (in-context dispatch cost)",
            # the same launches over every decode step of a whole generate: exit-to-exit spans in the production
            # chain (previous launch's last wave exit -> this launch's last wave exit: the boundary before the launch
            # instead of rocprof's after it), and the in-kernel wave spans alone
            "chain": chain,
            "in_kernel_waves": waves,
            "down_kernel": prof["moe_down_kernel"],
            "in_context": {k: ctx_line(k) for k in ("moe_gateup", "moe_down", "attention")},
            "moe_total": moe_total,
            "others": {k: {"avg_us": round(prof[k]["avg_us"], 2), "bytes": prof[k]["bytes"],
                           "GB/s": round(prof[k]["bytes"] / (prof[k]["avg_us"] * 1e-6) / 1e9, 1)}
                       for k in ("lm_head", "lm_head_screened", "qkv", "o_proj", "router")
                       if prof.get(k, {}).get("avg_us", 0) > 0},
            "layers_step_us": round(prof["layers_step"]["avg_us"], 1),
            "kv_len": prof["kv_len"]}


def main():
    if "--cpu-leg" in sys.argv:  # the all-CPU baseline leg's child process (cpu_baseline)
        return cpu_leg_child(sys.argv[sys.argv.index("--cpu-leg") + 1])
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--pages-per-gpu", type=int, default=1)
    ap.add_argument("--max-new-tokens", type=int, default=512)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-decode-steps", type=int, default=0, help="(unused: the C++ baseline times every decode step)")
    ap.add_argument("--roofline-iters", type=int, default=20)
    ap.add_argument("--no-chain-roofline", action="store_true",
                    help="skip the per-layer launch chain's roofline beside the persistent decode's (one page)")
    ap.add_argument("--trace-only", action="store_true",
                    help="production-only run for a rocprofv3 kernel trace: the timed generates and nothing else "
                         "(no span / event / profile_decode generates, no CPU baseline); roofline is null")
    ap.add_argument("--workload", default="deepseek", choices=["deepseek", "dots2048"],
                    help="deepseek: configs[1]/[2] (default); dots2048: configs[3], the dots.ocr vision tower")
    ap.add_argument("--dots-size", type=int, default=2048,
                    help="page side: 2048 (configs[3]) is resized to 2044 by smart_resize + the Catmull-Rom pass")
    ap.add_argument("--snapshot", default=None, choices=["q4k"],
                    help="q4k: configs[4], a full-size synthetic Q4_K DSQ snapshot loaded through the engine's "
                         "dequant-on-load path (written to $TMPDIR first)")
    ap.add_argument("--text-pages", action="store_true",
                    help="each page is a 706-token text prompt (dsocr.synth.text_page_prompt) instead of an image: "
                         "prefill + decode only; the pages decode distinct streams, so a batch routes its MoE layers "
                         "like distinct real pages (~35 experts per layer at 8 pages)")
    ap.add_argument("--oversubscribe", action="store_true",
                    help="allow more ranks than visible GPUs (ranks then share devices; n_gpus reports the "
                         "distinct devices used, `ranks` the rank count) - a test of the launch path only")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_under_torchrun(args.gpus))   # before any HIP call in this process
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != args.gpus:
        log(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per requested GPU")
        sys.exit(2)
    n_vis = max(1, visible_gpus())
    if world > n_vis and not args.oversubscribe:
        log(f"[bench] {world} ranks but {n_vis} visible GPU(s): refusing to share devices (--oversubscribe to test)")
        sys.exit(2)
    local = local % n_vis   # one GPU per rank; ranks share a GPU only under --oversubscribe
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")   # host-side barrier / max only; the data path has no collective
    devices = rank_devices(dist, local)
    n_dev = len(set(devices))

    if args.workload == "dots2048":
        res = run_dots(args, rank, world, local, dist)
        if res is not None:
            res.update(n_gpus=n_dev, ranks=world, devices=devices)
            print(json.dumps(res), flush=True)
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    import numpy as np

    import dsocr
    from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model
    from dsocr._lib import check, lib
    from dsocr.synth import BENCH_PROMPT, SyntheticTokenizer, synthetic_page, text_page_prompt

    def barrier():
        check(lib().dsocr_dev_sync())
        if dist is not None:
            dist.barrier()

    snap = None
    if args.snapshot == "q4k":
        import tempfile

        from dsocr.synth import write_synthetic_snapshot
        snap_path = os.path.join(tempfile.gettempdir(), f"dsocr_synth_q4k_r{rank}.dsq")
        t = time.time()
        snap = write_synthetic_snapshot(json.load(open(dsocr.FULL_CONFIG)), snap_path, seed=0)
        snap["write_s"] = round(time.time() - t, 1)
        log(f"[rank {rank}] synthetic Q4_K snapshot {snap} -> {snap_path}")
    t_load = time.time()
    eng = load_model(ModelLoadArgs(config_path=dsocr.FULL_CONFIG, synthetic_seed=0, dtype="f16", device=local,
                                   snapshot_path=snap_path if snap else None))
    load_s = time.time() - t_load
    log(f"[rank {rank}] engine loaded on hip:{local} in {load_s:.1f}s")
    if snap:
        snap["load_s"] = round(load_s, 1)
        os.unlink(snap_path)  # the engine holds the dequantised weights in HBM
    tok = SyntheticTokenizer(eng.vocab)
    vs = VisionSettings(1024, 640, True)
    ppg = args.pages_per_gpu

    prep_gpu_s = [0.0]

    def make_batch(step):
        imgs, reqs = [], []
        for idx in page_indices(step, world, rank, ppg):
            if args.text_pages:
                imgs.append(None)
                reqs.append((text_page_prompt(idx, vocab=eng.vocab), None, None, None))
                continue
            img = synthetic_page(idx)
            t0 = time.time()
            page = Page(img, vs, eng)   # a1-a3 on the GPU: pixels HBM-resident before the timed region
            prep_gpu_s[0] += time.time() - t0
            ids, mask = build_prompt_tokens(tok, BENCH_PROMPT, [page.n_image_tokens])
            imgs.append(img)
            reqs.append((ids, mask, page, None))
        return imgs, reqs

    params = DecodeParameters(max_new_tokens=args.max_new_tokens)
    batches = [make_batch(s) for s in range(args.warmup + args.steps)]
    gpu_prep_ms = prep_gpu_s[0] * 1e3 / max(1, len(batches) * ppg)
    t = time.time()
    if not args.text_pages:
        Page(synthetic_page(0), vs)  # the host C++ path on the same page, for the report
    prep_ms = (time.time() - t) * 1e3
    for s in range(args.warmup):
        eng.generate_batch(batches[s][1], params, ignore_eos=True)

    timings = []
    barrier()
    t0 = time.perf_counter()
    for s in range(args.warmup, args.warmup + args.steps):
        out = eng.generate_batch(batches[s][1], params, ignore_eos=True)
        assert all(len(o) == args.max_new_tokens for o in out)
        timings.append(eng.last_timings())
    barrier()
    elapsed = time.perf_counter() - t0
    iterative_s = sum(t["decode_iterative_ms"] for t in timings) / 1e3
    stage = {k: sum(t[k] for t in timings) / len(timings)
             for k in ("vision_compute_ms", "decode_prefill_ms", "decode_iterative_ms", "vision_flops", "prefill_flops")}
    tokens_rank = args.steps * ppg * args.max_new_tokens
    tok_s_rank = tokens_rank / iterative_s if iterative_s > 0 else 0.0
    elapsed, tok_s = reduce_over_ranks(dist, elapsed, tok_s_rank)
    pages_total = args.steps * ppg * world
    value = pages_total / elapsed

    result = None
    if rank == 0:
        log(f"[bench] timed: {value:.4f} pages/s, {tok_s:.1f} decode tok/s, stages "
            + ", ".join(f"{k} {stage[k]:.2f}" for k in ("vision_compute_ms", "decode_prefill_ms", "decode_iterative_ms")))
        roofline = None
        if not args.trace_only:
            if eng.persist_info()["used"] and ppg == 1:  # the timed generates ran the persistent decode
                roofline = persist_roofline(eng, batches[args.warmup][1], params, ppg, args)
                if not args.no_chain_roofline:  # the per-layer launch chain's line, same page (DSOCR_PERSIST=0)
                    os.environ["DSOCR_PERSIST"] = "0"
                    roofline["launch_chain"] = decode_roofline(eng, batches[args.warmup][1], params, ppg, args)
                    os.environ.pop("DSOCR_PERSIST")
            else:
                roofline = decode_roofline(eng, batches[args.warmup][1], params, ppg, args)
        cpu = None
        if world == 1 and not (args.no_cpu_baseline or args.trace_only) and not snap and not args.text_pages:
            b = batches[args.warmup]
            try:
                cpu = cpu_baseline(b[0], b[1][0][0], b[1][0][1], args.max_new_tokens, args.cpu_decode_steps)
            except Exception as e:  # reported, not fatal for the GPU number
                cpu = {"value": None, "error": repr(e)}
        result = {
            "metric": "pages/sec + decode tok/s, DeepSeek-OCR fp16 1024px/512tok",
            "value": round(value, 4),
            "unit": "pages/s",
            "decode_tok_s": round(tok_s, 1),
            "n_gpus": n_dev,       # distinct devices the ranks ran on (== ranks unless --oversubscribe)
            "ranks": world,
            "devices": devices,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("f32 (Q4_K / Q8_0 snapshot linears dequantised to fp16 at load)" if snap else
                      "f32 (fp16-rounded decoder weights, bf16 vision/lm_head weights)"),
            "data": "synthetic 1024x1024 pages + seeded synthetic weights (no checkpoint offline)"
                    + ("; snapshot linears: random valid Q4_K / Q8_0 blocks" if snap else ""),
            "config": {"workload": ("configs[4]: deepseek-ocr-q4k DSQ snapshot, dequant-on-load -> fp16 kernels, "
                                    f"{ppg} pages/GPU batch") if snap else
                                   (f"deepseek-ocr, {ppg} text pages/GPU: 706-token text prompts (no vision), 512 "
                                    "greedy tokens, distinct decode streams per page" if args.text_pages else
                                    "configs[1]: deepseek-ocr, 1024x1024 page, crop (2,2), 706-token prefill, "
                                    "512 greedy tokens" if ppg == 1 else f"deepseek-ocr, {ppg} pages/GPU batch"),
                       "pages_per_gpu": ppg, "global_batch": ppg * world, "prefill_tokens": len(batches[0][1][0][0]),
                       "max_new_tokens": args.max_new_tokens, "parallelism": f"dp{world}"},
            "stage_ms": {k: round(stage[k], 2) for k in ("vision_compute_ms", "decode_prefill_ms", "decode_iterative_ms")},
            # MFMA roofline of the compute-bound stages: algorithmic f32 FLOPs (engine-counted: linears 2MNK,
            # attention 4 Lq Lk d per head, causal prefill the lower triangle) / stage time, against the
            # dense bf16 MFMA peak the split-plane GEMMs run on; the exact-f32 contract issues each linear
            # as 3 (vision, bf16 weights) or 5 (prefill, f16 weights) bf16 planes, so `issued_frac` = plane
            # count x frac for the linears (the attention runs on the f32 MFMA / 3 bf16 planes of P)
            "roofline_mfma": {
                stg: {"bound": "mfma", "achieved": round(fl / (ms * 1e-3) / 1e12, 1), "peak": 2500.0,
                      "unit": "TFLOP/s", "frac": round(fl / (ms * 1e-3) / 1e12 / 2500.0, 4),
                      "issued_frac": round(planes * fl / (ms * 1e-3) / 1e12 / 2500.0, 4),
                      "tflop_per_page": round(fl / ppg / 1e12, 3), "ms_per_batch": round(ms, 2)}
                for stg, fl, ms, planes in (("vision", stage["vision_flops"], stage["vision_compute_ms"], 3),
                                            ("prefill", stage["prefill_flops"], stage["decode_prefill_ms"], 5))
                if fl > 0 and ms > 0},
            "snapshot": snap,
            "host_prepare_ms_per_page": round(prep_ms, 2),
            "gpu_prepare_ms_per_page": round(gpu_prep_ms, 2),
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
