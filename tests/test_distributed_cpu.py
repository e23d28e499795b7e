"""World-size-2/3 gloo tests of the multi-GPU path on CPU: shard ranges, the block-sum
all-gather and the fixed-order total (bitwise identical to one process).  The exchange
under test is shard.BlockExchange, the code bench.py's N > 1 branch runs each step; the
block sums come from the oracle's per-pattern lnL of a real workload shard (what each
rank's plk_evaluate returns on the GPU)."""
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


def _oracle_sites(config, start, end):
    import oracle
    import workload

    wl = workload.make_workload(config, n_patterns=end)
    et = wl.et
    states = wl.simulate(start, end).astype(np.int32)
    pm = np.zeros((et.n_nodes, wl.C, wl.S, wl.S))
    for n in range(et.n_nodes):
        if n != et.root:
            m = wl.models[0] if wl.model_of_node is None else wl.models[wl.model_of_node[n]]
            for c in range(wl.C):
                pm[n, c] = m.pij(et.brlen[n] * wl.rates[c])
    ss, sons, lr = et.son_arrays()
    _, site, _, _ = oracle.tree_loglik(ss, sons, lr, et.root, states, wl.alphabet.init_table, pm, wl.probs,
                                       wl.root_freqs, use_patterns=False, scaling=wl.scaling, want_sites=True)
    return site


def _bench_worker(rank, world, port, config, n, q, scaling="strong"):
    """bench.py's N > 1 exchange: each rank holds its shard's block sums (its range from
    shard.bench_range, as bench.py computes it), BlockExchange (sized once at setup)
    all-gathers them and sums in global block order."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b, _ = shard.bench_range(scaling, rank, world, n)
    site = _oracle_sites(config, a, b)
    blocks = _block_sums(np.concatenate([np.zeros(a), site]), a, b)   # block sums of [a, b)
    x = shard.BlockExchange(dist, len(blocks), device="cpu")
    lnl1 = x.lnl(blocks)
    lnl2 = x.lnl(blocks)        # a second evaluation reuses the buffers
    q.put((rank, lnl1, lnl2))
    dist.destroy_process_group()


@pytest.mark.parametrize("config,world,n,scaling", [("gtr_g4_dna_1M_64", 2, 3 * 4096 + 300, "strong"),
                                                    ("nh_gtr_g4_dna_2M_512", 3, 2 * 4096 + 5, "strong"),
                                                    ("nh_gtr_g4_dna_2M_512", 2, 5 * 4096, "strong"),
                                                    ("gtr_g4_dna_1M_64", 3, 900, "strong"),
                                                    ("gtr_g4_dna_1M_64", 2, 2 * 4096, "weak")])
def test_block_exchange_bitwise_vs_one_process(config, world, n, scaling):
    """bench.py's N > 1 path in both scaling modes: strong (config 5's global pattern count
    split over the ranks; the lnL is bitwise the one-process total) and weak (each rank its
    own block-aligned slice; the total is that of the union)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, config, n, q, scaling)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    total = shard.bench_range(scaling, 0, world, n)[2]
    whole = shard.fixed_order_sum(_block_sums(_oracle_sites(config, 0, total), 0, total))
    assert all(r[1] == whole and r[2] == whole for r in res), (res, whole)


def test_bench_range_modes():
    """Strong: contiguous block-aligned ranges tiling the job's patterns (config 5: 2M over
    1/2/4/8 ranks); weak: one slice per rank."""
    for world in (1, 2, 3, 4, 8):
        rs = [shard.bench_range("strong", r, world, 2_000_000) for r in range(world)]
        assert rs[0][0] == 0 and rs[-1][1] == 2_000_000 and all(r[2] == 2_000_000 for r in rs)
        assert all(a[1] == b[0] and b[0] % shard.BLOCK == 0 for a, b in zip(rs, rs[1:]))
        assert max(r[1] - r[0] for r in rs) - min(r[1] - r[0] for r in rs) <= 2 * shard.BLOCK
        ws = [shard.bench_range("weak", r, world, 1_000_000) for r in range(world)]
        assert ws[-1] == ((world - 1) * 1_000_000, world * 1_000_000, world * 1_000_000)


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


_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_stdout_is_one_json_line(tmp_path):
    """Under torch.distributed.run every rank's stdout reaches the driver: RCCL prints a version
    banner and gloo its connection messages on fd 1.  bench.py moves fd 1 to stderr at start
    and writes only rank 0's JSON line to the original stdout (bench._json_stdout)."""
    import subprocess
    import sys
    code = (
        "import importlib.util, os, sys\n"
        f"spec = importlib.util.spec_from_file_location('bench', {os.path.join(_REPO, 'bench.py')!r})\n"
        "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n"
        "out = b._json_stdout()\n"
        "print('python-level noise'); os.write(1, b'C-level banner\\n')\n"
        "print('{\"metric\": \"m\"}', file=out, flush=True)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ['{"metric": "m"}']
    assert "C-level banner" in r.stderr and "python-level noise" in r.stderr


# ---------------------------------------------------------------- libplk's own exchange bookkeeping

def _exchange_worker(rank, world, port, counts, flags, n_deriv, q):
    """One rank of plk_comm_init's exchange with gloo standing in for RCCL: its record packed
    by libplk (plk_exchange_pack), the fixed-size all-gather, then libplk's reduction
    (plk_exchange_reduce) and rank-order derivative sums (plk_exchange_rank_sums) -- the code
    root_finish / comm_sum_values run on the gathered buffers."""
    import torch
    import plk
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blocks_all, deriv_all = _exchange_data(counts, world, n_deriv)
    a = sum(counts[:rank])
    mine = blocks_all[a:a + counts[rank]]
    # the block counts are exchanged once, as plk_comm_init does
    cnt = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(cnt, torch.tensor([len(mine)], dtype=torch.int64))
    got_counts = [int(c.item()) for c in cnt]
    stride = plk.exchange_stride(got_counts)
    rec = plk.exchange_pack(mine, flags[rank], stride)
    parts = [torch.zeros(stride, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(parts, torch.from_numpy(rec))
    gathered = torch.stack(parts).numpy()
    lnl, uflow = plk.exchange_reduce(gathered, got_counts, stride)
    dv = [torch.zeros(n_deriv, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(dv, torch.from_numpy(deriv_all[rank].copy()))
    d = plk.exchange_rank_sums(torch.stack(dv).numpy(), world)
    q.put((rank, got_counts, stride, rec.tolist(), lnl, uflow, d.tolist()))
    dist.destroy_process_group()


def _exchange_data(counts, world, n_deriv):
    """Block sums over a wide dynamic range, so that any other order of adds changes the
    total's low bits; per-rank derivative sums likewise."""
    rng = np.random.default_rng(sum(counts) * 31 + world)
    blocks = -rng.gamma(2.0, 1.0, size=sum(counts)) * 10.0 ** rng.uniform(-2, 7, size=sum(counts))
    deriv = rng.normal(size=(world, n_deriv)) * 10.0 ** rng.uniform(-3, 6, size=(world, n_deriv))
    return blocks, deriv


@pytest.mark.parametrize("counts,flags", [
    ([5, 3], [0, 0]),                    # the last rank has fewer blocks than the widest
    ([2, 7, 4], [0, 1, 0]),              # a flag on a middle rank reaches every rank
    ([245, 245, 245, 245, 245, 245, 245, 244], [0] * 7 + [1]),   # config 5's 2 M over 8 ranks
    ([9, 1, 1, 6, 3, 8, 2, 1], [0] * 8),  # ragged, world 8
    ([1, 0, 4], [0, 0, 0])])             # a rank with no blocks
def test_libplk_exchange_multi_rank_bitwise(counts, flags):
    """libplk's exchange bookkeeping at world 2 / 3 / 8 over gloo with uneven per-rank block
    counts (padding to the widest rank's count): every rank gets the one-process fixed-order
    sum of all blocks bitwise (RNonHomogeneousTreeLikelihood.cpp:168-182 summed as one chain),
    the OR of the underflow flags, and the rank-order derivative sums; the record is the
    documented layout (block sums, zeros, flag)."""
    world = len(counts)
    n_deriv = 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, counts, flags, n_deriv, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    blocks, deriv = _exchange_data(counts, world, n_deriv)
    whole = 0.0
    for b in blocks:          # one process over every block, block order
        whole += b
    dsum = np.zeros(n_deriv)
    for r in range(world):    # rank order
        dsum = dsum + deriv[r]
    stride = max(counts) + 1
    a = 0
    for rank, got_counts, st, rec, lnl, uflow, d in res:
        assert got_counts == counts and st == stride
        exp_rec = list(blocks[a:a + counts[rank]]) + [0.0] * (stride - 1 - counts[rank]) + [float(flags[rank])]
        assert rec == exp_rec
        a += counts[rank]
        assert lnl == whole, (rank, lnl, whole)
        assert uflow == any(flags)
        assert np.array_equal(np.array(d), dsum)


def test_libplk_exchange_argument_checks():
    import plk
    with pytest.raises(plk.PlkError):
        plk.exchange_stride([3, -1])
    with pytest.raises(plk.PlkError):
        plk.exchange_pack(np.ones(4), False, 4)             # 4 blocks + the flag need stride 5
    with pytest.raises(plk.PlkError):
        plk.exchange_reduce(np.zeros((2, 3)), [2, 3], 3)    # rank 1's 3 blocks exceed its record
