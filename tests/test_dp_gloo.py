"""Whole-graph data parallelism on CPU (gloo, world_size 2 and 4): the Trainer's DP
bookkeeping (sgnn_amd.train.DataParallel: N_global count, 1/N_global loss
scaling, SUM all-reduce of one flat gradient buffer) must reproduce the
single-process gradient of the concatenated batch (train.py:268 takes the
mean over all particles of the batch).  Gradients come from the oracle here
(no GPU); on MI355X the same DataParallel object all-reduces over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import golden, state_of, stats_of


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


GRAPH_DIMS = [(10, 8), (12, 7), (9, 9), (11, 6)]   # unequal graph sizes


def _graphs():
    from sgnn_amd import synthetic
    from oracle import sgnn_oracle as O
    out = []
    for k, (nx, ny) in enumerate(GRAPH_DIMS):
        seq = synthetic.trajectory(synthetic.lattice_2d(nx, ny), 12, seed=50 + k)
        pos, nxt = torch.from_numpy(seq[:, :11]), torch.from_numpy(seq[:, 11])
        strain = torch.from_numpy(np.random.default_rng(k).normal(0, 1, seq.shape[0]).astype(np.float32))
        noise = O.random_walk_noise(pos, 0.02, generator=torch.Generator().manual_seed(9 + k))
        out.append((pos, nxt, strain, noise))
    return out


def _oracle_grads(graphs, inv_count):
    """sum over graphs of d/dtheta [ inv_count * sum_particles loss_i ]"""
    from oracle import sgnn_oracle as O
    z = golden("train2d_r06")
    state = {k: v.clone().requires_grad_(True) for k, v in state_of(z, "w0/").items()}
    sim = O.OracleSimulator(state, 2, 5, 0.6, stats_of(z))
    sim.p = state
    total = 0.0
    for pos, nxt, strain, noise in graphs:
        n = pos.shape[0]
        pa, ta, ps = sim.predict_accelerations(nxt, noise, pos, [n], torch.zeros(n, dtype=torch.long))
        loss_sum = O.training_loss(pa, ta, ps, strain) * n       # sum over this graph's particles
        (loss_sum * inv_count).backward()
        total += float(loss_sum)
    names = [k for k in state if state[k].grad is not None]
    flat = torch.cat([state[k].grad.reshape(-1) for k in names])
    return flat, total * inv_count


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sgnn_amd.train import DataParallel
    from sgnn_amd.train import split_batch
    dp = DataParallel()
    mine = [_graphs()[i] for i in split_batch(list(range(len(GRAPH_DIMS))), rank, world)]   # contiguous shares
    n_local = sum(g[0].shape[0] for g in mine)
    n_global = dp.global_count(n_local, "cpu")
    flat, loss = _oracle_grads(mine, 1.0 / n_global)
    loss_t = torch.tensor([loss])
    dp.allreduce_(flat, loss_t)
    q.put((rank, n_global, flat.numpy(), float(loss_t)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_whole_graph_dp_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    graphs = _graphs()
    n_total = sum(g[0].shape[0] for g in graphs)
    ref_flat, ref_loss = _oracle_grads(graphs, 1.0 / n_total)
    for rank, n_global, flat, loss in res:
        assert n_global == n_total
        np.testing.assert_allclose(flat, ref_flat.numpy(), rtol=1e-4, atol=1e-7)
        assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss)
    # every rank ends with the identical gradient -> identical Adam update
    for r in res[1:]:
        np.testing.assert_array_equal(res[0][2], r[2])


def _deferred_worker(rank, world, port, q):
    """The sync-free DP step (DataParallel.plan / put_count / take_count, what Trainer.train_step does when
    the caller passes no n_global): no all_gather, the gradient of this rank's loss SUM and its particle
    count go through ONE sum all-reduce, the count scales the reduced gradient afterwards."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sgnn_amd.train import DataParallel, split_batch

    def no_gather(*a, **k):
        raise AssertionError("the deferred DP step must not gather the counts")
    dist.all_gather = no_gather
    dp = DataParallel()
    mine = [_graphs()[i] for i in split_batch(list(range(len(GRAPH_DIMS))), rank, world)]
    n_local = sum(g[0].shape[0] for g in mine)
    inv, off, deferred = dp.plan(n_local, None, None)
    assert deferred and inv == 1.0 and off == rank * DataParallel.RANK_NOISE_STRIDE
    flat, loss = _oracle_grads(mine, inv)
    comm = torch.zeros(flat.numel() + 8)
    comm[:flat.numel()] = flat
    tail = comm[flat.numel():]
    tail[0] = loss
    dp.put_count(tail, n_local)
    dp.allreduce_(comm)
    n_global = dp.take_count(comm[:flat.numel()], tail)
    q.put((rank, int(n_global), comm[:flat.numel()].numpy().copy(), float(tail[0] / n_global)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_deferred_count_dp_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_deferred_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    graphs = _graphs()
    n_total = sum(g[0].shape[0] for g in graphs)
    ref_flat, ref_loss = _oracle_grads(graphs, 1.0 / n_total)
    for rank, n_global, flat, loss in res:
        assert n_global == n_total
        np.testing.assert_allclose(flat, ref_flat.numpy(), rtol=1e-4, atol=1e-7)
        assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss)
    for r in res[1:]:
        np.testing.assert_array_equal(res[0][2], r[2])


def test_count_slots_are_exact_for_large_counts():
    """put_count splits the count into two float slots (hi * 2^20 + lo), so the summed count stays
    exact in fp32 far past 2^24 particles (C5: 8 ranks x ~1 M)."""
    from sgnn_amd.train import DataParallel
    dp = DataParallel()
    tails = []
    for n in (1_000_003, 999_999_937, 5, (1 << 40) + 12345):
        t = torch.zeros(8)
        dp.put_count(t, n)
        tails.append((n, t))
    tot = torch.zeros(8)
    for _, t in tails:
        tot += t
    g = torch.ones(4)
    cnt = dp.take_count(g, tot)
    n_sum = sum(n for n, _ in tails)
    assert int(tot[6].double() * 2 ** 20 + tot[7].double()) == n_sum
    assert abs(float(cnt) - n_sum) <= 1e-7 * n_sum


def _layout_worker(rank, world, port, q):
    """Ragged, changing per-rank counts: rank 0 repeats n, rank 1 changes it
    every step.  Every step = layout (one all_gather) + one gradient-sized
    all_reduce; a rank-local cache would pair different collectives here."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sgnn_amd.train import DataParallel
    dp = DataParallel()
    seen = []
    for step in range(6):
        n_local = 100 if rank == 0 else 50 + 7 * step
        n_global, offset = dp.layout(n_local, "cpu")
        g = torch.full((1000,), float(rank + 1))
        dp.allreduce_(g)
        seen.append((n_global, offset, float(g[0])))
    q.put((rank, seen))
    dist.destroy_process_group()


def test_layout_never_desyncs_with_ragged_changing_counts():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_layout_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for step in range(6):
        n1 = 50 + 7 * step
        assert res[0][step] == (100 + n1, 0, 3.0)
        assert res[1][step] == (100 + n1, 100, 3.0)


def test_split_batch_contiguous_balanced_and_skips_short_batches():
    from sgnn_amd.train import split_batch
    for n, world in ((8, 8), (8, 3), (7, 2), (5, 4), (2, 2)):
        idx = list(range(100, 100 + n))
        parts = [split_batch(idx, r, world) for r in range(world)]
        assert sum(parts, []) == idx                       # rank order = concatenation order
        sizes = [len(p) for p in parts]
        assert max(sizes) - min(sizes) <= 1 and min(sizes) >= 1
    # an epoch's short last batch (fewer graphs than ranks): every rank skips it
    assert all(split_batch([3], r, 2) is None for r in range(2))
    assert split_batch([3], 0, 1) == [3]


def test_dp_epoch_with_odd_sample_count_has_matching_collectives():
    """train()'s batching at world 2, batch_size 2 and an odd sample count: the
    last batch holds 1 graph; both ranks must skip it (no rank left waiting
    in a collective), and every other batch feeds both ranks."""
    from sgnn_amd.train import split_batch
    g = torch.Generator().manual_seed(0)
    sampler = torch.utils.data.RandomSampler(range(9), generator=g)
    batches = list(torch.utils.data.BatchSampler(sampler, 2, drop_last=False))
    plans = [[split_batch(b, r, 2) for b in batches] for r in range(2)]
    steps = [[p is not None for p in plan] for plan in plans]
    assert steps[0] == steps[1]                            # same number of collectives per rank
    assert steps[0].count(False) == 1 and steps[0][-1] is False


def test_layer_buckets_tile_the_flat_gradient():
    """The overlapped data-parallel all-reduce sends each interaction layer's
    gradient slice as soon as its slab reduction is queued, then [0, lo) and
    [hi, end): the buckets must be contiguous, disjoint, in layer order, and
    cover the flat buffer (gradients + loss tail) exactly once."""
    import torch
    from sgnn_amd import synthetic, training
    from sgnn_amd.learned_simulator import LearnedSimulator
    from sgnn_amd.train import layer_ranges
    st = synthetic.normalization_stats(2, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    for ntypes, emb in ((1, 9), (3, 4)):
        sim = LearnedSimulator(2, 21 + (emb if ntypes > 1 else 0), 3, 64, 5, 1, 64, 0.6, stats, ntypes, emb)
        flat = training.FlatParams(sim)
        ranges, (lo, hi) = layer_ranges(sim._encode_process_decode, flat)
        assert len(ranges) == 5 and ranges[0][0] == lo and ranges[-1][1] == hi
        for (s0, e0), (s1, e1) in zip(ranges, ranges[1:]):
            assert e0 == s1 and s0 < e0
        cover = torch.zeros(flat.comm.numel(), dtype=torch.int32)
        for s, e in [(0, lo)] + ranges + [(hi, flat.comm.numel())]:
            cover[s:e] += 1
        assert bool((cover == 1).all())
        # every processor parameter's gradient view lies inside its own layer's bucket
        for k, layer in enumerate(sim._encode_process_decode._processor.gnn_stacks):
            for p in layer.parameters():
                off, n = flat.offsets[id(p)]
                assert ranges[k][0] <= off and off + n <= ranges[k][1]


def test_block_buckets_tile_the_flat_gradient():
    """The multi-scale trainer's overlapped buckets (train.block_buckets): one
    per G2M / M2M / M2G block in chain order, plus the intervals no block
    covers (encoders, head, loss sums); together they cover the flat buffer
    exactly once and every block parameter lies in its own block's bucket."""
    import torch
    from sgnn_amd import synthetic, training
    from sgnn_amd.multi_scale import MultiScaleSimulator
    from sgnn_amd.train import block_buckets
    st = synthetic.normalization_stats(2, noise_std=0.02)
    stats = {k: {kk: torch.from_numpy(vv) for kk, vv in v.items()} for k, v in st.items()}
    sim = MultiScaleSimulator(2, 11, 3, 64, 64, 3, 2, stats, 1, 9, 2, 2, 2.0)
    flat = training.FlatParams(sim)
    blocks = sim._multi_scale_gnn.chain()
    ranges, rest = block_buckets(blocks, flat)
    assert len(ranges) == len(blocks) == 5 and rest
    cover = torch.zeros(flat.comm.numel(), dtype=torch.int32)
    for s, e in ranges + rest:
        assert s < e
        cover[s:e] += 1
    assert bool((cover == 1).all())
    for b, blk in enumerate(blocks):
        for p in blk.parameters():
            off, n = flat.offsets[id(p)]
            assert ranges[b][0] <= off and off + n <= ranges[b][1]
