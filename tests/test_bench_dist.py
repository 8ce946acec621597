"""The N>1 bench path on CPU: world_size-2 gloo ranks (the data path has no collective;
only the barrier and the max-over-ranks / sum reductions go through torch.distributed)."""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pages = [bench.page_indices(s, world, rank, 8) for s in range(3)]
    elapsed, tok_s = bench.reduce_over_ranks(dist, 1.0 + rank, 100.0 * (rank + 1))
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, pages, elapsed, tok_s))


def test_page_sharding_single_rank():
    assert bench.page_indices(0, 1, 0, 1) == [0]
    assert bench.page_indices(2, 1, 0, 8) == list(range(16, 24))
    assert bench.reduce_over_ranks(None, 2.5, 7.0) == (2.5, 7.0)


@pytest.mark.timeout(120)
def test_two_rank_gloo_sharding_and_reduction():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=90) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    all_pages = [i for _, pages, _, _ in res for step in pages for i in step]
    assert len(all_pages) == len(set(all_pages)) == 2 * 3 * 8      # disjoint, nothing dropped
    assert sorted(all_pages) == list(range(48))
    for _, _, elapsed, tok_s in res:
        assert elapsed == 2.0          # max over ranks
        assert tok_s == 300.0          # sum over ranks


def test_world_size_must_match_gpus():
    """A launcher's WORLD_SIZE that disagrees with --gpus is refused before any device work."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 2 and "WORLD_SIZE=2 but --gpus 1" in out.stderr


@pytest.mark.timeout(300)
def test_gpus_flag_launches_ranks_and_refuses_shared_devices():
    """`bench.py --gpus 2` with no launcher starts two ranks under torch.distributed.run; with fewer
    visible GPUs than ranks (none here) every rank refuses to share a device, so the run exits non-zero
    and prints no JSON line instead of reporting shared-device throughput as 2 GPUs."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"], cwd=ROOT,
                         env=env, capture_output=True, text=True, timeout=280)
    assert out.returncode != 0
    assert "without a launcher" in out.stderr and "refusing to share devices" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_two_rank_bench_process_run(gpu):
    """`python bench.py --gpus 2` exactly as a user types it (no launcher): the bench re-launches itself under
    torch.distributed.run (one process per rank, gloo barrier and max-over-ranks timing).  The box has one
    GPU, so --oversubscribe lets both engines share it: one JSON line from rank 0 whose value counts both
    ranks' pages, ranks == 2, and n_gpus == the distinct devices actually used."""
    import json
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--oversubscribe", "--steps", "1",
           "--warmup", "0", "--max-new-tokens", "8", "--no-cpu-baseline", "--roofline-iters", "1"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "4"
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["ranks"] == 2 and len(res["devices"]) == 2 and res["n_gpus"] == len(set(res["devices"]))
    assert res["config"]["global_batch"] == 2 and res["value"] > 0
    assert abs(res["value"] - 2 / (res["ms_per_step"] / 1e3)) < 1e-3 * res["value"] + 1e-3


def test_span_roofline_prices_each_launch():
    """bench.span_roofline: every recorded launch priced from its own expert count (gate/up, down) or
    step (attention), achieved = sum(bytes) / sum(durations); empty slots ignored."""
    import numpy as np
    d = bench.lang_dims({"hidden_size": 1280, "moe_intermediate_size": 896, "n_shared_experts": 2,
                         "num_experts_per_tok": 6, "num_attention_heads": 10, "num_key_value_heads": 10})
    arr = np.zeros((3, 12, 8, 5), np.uint64)
    # gate/up, layer 1: steps 1 and 2, 9 us and 11 us (900 / 1100 ticks of 10 ns), 6 and 30 experts
    arr[0, 1, 1] = [1000, 1900, 6, 7168, 9000]
    arr[0, 1, 2] = [5000, 6100, 30, 7168, 11000]
    # attention, layer 0, step 3: 8 us
    arr[2, 0, 3] = [100, 900, 0, 800, 8000]
    got = bench.span_roofline({"moe_gateup": arr[0], "moe_down": arr[1], "attention": arr[2]}, d, 8, 706)
    assert set(got) == {"moe_gateup", "attention"}
    g = got["moe_gateup"]
    b6 = bench.span_bytes("moe_gateup", d, 8, 706, 6, 1)
    b30 = bench.span_bytes("moe_gateup", d, 8, 706, 30, 2)
    assert b30 - b6 == 24 * 2 * 896 * 1280 * 2
    assert g["launches"] == 2 and abs(g["avg_us"] - 10.0) < 1e-9 and abs(g["wave_avg_us"] - 10.0) < 1e-9
    assert g["timing"] == "hip events in graph"
    assert abs(g["GB/s"] - (b6 + b30) / 20e-6 / 1e9) < 1e-6 and g["experts_range"] == [6, 30]
    a = got["attention"]
    assert abs(a["GB/s"] - bench.span_bytes("attention", d, 8, 706, 0, 3) / 8e-6 / 1e9) < 1e-6
    assert bench.span_bytes("attention", d, 1, 706, 0, 3) == 709 * 10 * 128 * 8 + (3840 + 1280) * 4


def test_chain_roofline_exit_to_exit():
    """bench.chain_roofline: a launch's duration = its last wave exit - the previous launch's last exit (router ->
    gate/up -> down, attention -> o_proj -> router, down of layer l - 1 -> attention of l at one page), boundary =
    its first entry - that exit; MoE launches priced at the wave-span generate's expert counts."""
    import numpy as np
    d = bench.lang_dims({"hidden_size": 1280, "moe_intermediate_size": 896, "n_shared_experts": 2,
                         "num_experts_per_tok": 6, "num_attention_heads": 10, "num_key_value_heads": 10})
    K = ("moe_gateup", "moe_down", "attention", "o_proj", "router")
    ch = {k: np.zeros((3, 4, 5), np.uint64) for k in K}
    wv = {k: np.zeros((3, 4, 5), np.uint64) for k in K[:3]}
    # layer 1, step 2 (100 MHz ticks): attention [0, 1100], o_proj [1250, 1500], router [1650, 1900],
    # gate/up [2050, 2800], down [2950, 3600]; layer 2 attention [3750, 4800]
    for k, (e, x) in {"attention": (0, 1100), "o_proj": (1250, 1500), "router": (1650, 1900),
                      "moe_gateup": (2050, 2800), "moe_down": (2950, 3600)}.items():
        ch[k][1, 2, 0], ch[k][1, 2, 1] = e, x
    ch["attention"][2, 2, 0], ch["attention"][2, 2, 1] = 3750, 4800
    wv["moe_gateup"][1, 2, 2] = 6
    wv["moe_down"][1, 2, 2] = 6
    got = bench.chain_roofline(ch, wv, d, 1, 706)
    g = got["moe_gateup"]
    assert g["launches"] == 1 and abs(g["avg_us"] - 9.0) < 1e-9 and abs(g["boundary_us"] - 1.5) < 1e-9
    assert abs(g["wave_us"] - 7.5) < 1e-9
    assert g["bytes_per_launch"] == bench.span_bytes("moe_gateup", d, 1, 706, 6, 2)
    assert abs(got["moe_down"]["avg_us"] - 8.0) < 1e-9
    assert abs(got["router"]["avg_us"] - 4.0) < 1e-9 and abs(got["o_proj"]["avg_us"] - 4.0) < 1e-9
    assert got["attention"]["launches"] == 1 and abs(got["attention"]["avg_us"] - 12.0) < 1e-9
    # 8 pages: the attention follows an unstamped q/k/v launch and is not priced
    assert "attention" not in bench.chain_roofline(ch, wv, d, 8, 706)
