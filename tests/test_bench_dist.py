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


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_two_rank_bench_process_run(gpu):
    """The N>1 bench as the driver launches it (torch.distributed.run, one process per rank, gloo barrier
    and max-over-ranks timing), two engines here sharing the box's one GPU (rank r uses GPU r % count):
    one JSON line from rank 0 whose value counts both ranks' pages."""
    import json
    import subprocess
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--max-new-tokens", "8", "--no-cpu-baseline",
           "--roofline-iters", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 2 and res["value"] > 0
    assert abs(res["value"] - 2 / (res["ms_per_step"] / 1e3)) < 1e-3 * res["value"] + 1e-3
