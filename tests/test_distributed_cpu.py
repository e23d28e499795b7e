"""World-size-2 gloo tests of the multi-GPU path on CPU: shard ranges, the block-sum
all-gather and the fixed-order total (bitwise identical to one process)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _site_lnl(n):
    rng = np.random.default_rng(7)
    return -rng.gamma(3.0, 20.0, size=n)


def _block_sums(site, start, end):
    out = []
    for b in range(start, end, shard.BLOCK):
        s = 0.0
        for v in site[b:min(b + shard.BLOCK, end)]:
            s += v
        out.append(s)
    return np.array(out)


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    site = _site_lnl(n)
    a, b = shard.shard_range(rank, world, n)
    lnl = shard.allgather_lnl(_block_sums(site, a, b), dist)
    q.put((rank, a, b, lnl))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 3 * 4096 + 17), (2, 100), (3, 10 * 4096)])
def test_gloo_allgather_bitwise(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    site = _site_lnl(n)
    ref = shard.fixed_order_sum(_block_sums(site, 0, n))
    assert all(r[3] == ref for r in res)
    # ranges tile [0, n) and are block aligned
    assert res[0][1] == 0 and res[-1][2] == n
    for (r0, a0, b0, _), (r1, a1, b1, _) in zip(res, res[1:]):
        assert b0 == a1 and (a1 % shard.BLOCK == 0 or a1 == n)


def test_shard_range_properties():
    for n in (1, 4095, 4096, 4097, 1_000_000, 2_000_000):
        for world in (1, 2, 4, 8):
            rs = [shard.shard_range(r, world, n) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a % shard.BLOCK == 0 or a == n for a, _ in rs)
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
