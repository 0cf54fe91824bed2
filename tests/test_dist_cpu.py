"""world_size-2 gloo tests of the multi-GPU plumbing (CPU)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from wespeaker_hubert_amd.dist import allreduce_sums, shard_bounds, shard_lines


def test_shard_split_matches_extract_embedding_sh():
    lines = [f"l{i}" for i in range(10)]
    # split -l $((10/4+1)) -> 3 lines per part: 3,3,3,1
    parts = [shard_lines(lines, r, 4) for r in range(4)]
    assert [len(p) for p in parts] == [3, 3, 3, 1]
    assert sum(parts, []) == lines
    assert shard_bounds(0, 0, 8) == (0, 0)
    for n in (1, 7, 64, 4874):
        for w in (1, 2, 3, 8):
            got = sum((shard_lines(list(range(n)), r, w) for r in range(w)), [])
            assert got == list(range(n))


def _worker(rank, world, port, x, g, n_groups, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_bounds(len(x), rank, world)
    acc = torch.zeros(n_groups, x.shape[1], dtype=torch.float64)
    cnt = torch.zeros(n_groups, dtype=torch.float64)
    xs = torch.from_numpy(x[lo:hi]).double()
    acc.index_add_(0, torch.from_numpy(g[lo:hi]).long(), xs)
    cnt.index_add_(0, torch.from_numpy(g[lo:hi]).long(), torch.ones(hi - lo, dtype=torch.float64))
    allreduce_sums(acc, cnt)
    q.put((rank, (acc / cnt.clamp(min=1).unsqueeze(1)).numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_cohort_allreduce_world2():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((101, 16)).astype(np.float32)
    g = rng.integers(0, 7, 101).astype(np.int32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, x, g, 7, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    ref = np.stack([x[g == i].astype(np.float64).mean(0) for i in range(7)])
    for r in range(2):
        np.testing.assert_allclose(res[r], ref, atol=1e-12)
