"""Multi-rank logic of bench.py on the CPU (gloo, world_size 2): the batch split, the
per-rank synthetic inputs and the only collectives (MAX of time, SUM of status counts).
The solve itself needs the GPU; everything a rank does around it is covered here."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from rmpc import workloads as W


def test_shard_covers_batch_exactly():
    for B, world in [(65536 * 8, 8), (262144, 8), (10, 3), (7, 4)]:
        cov = np.zeros(B, np.int32)
        for r in range(world):
            lo, hi = W.shard(B, world, r)
            cov[lo:hi] += 1
        assert np.all(cov == 1)


def test_round_robin_shards_cover_batch_and_match_global_inputs():
    """bench.py's split: rank r owns robots r, r + W, ...; its locally generated offsets and
    noise equal the single-process workload at those indices (no scatter needed)."""
    for B, world in [(65536 * 8, 8), (3 * 65536 + 1000, 4), (10, 3)]:
        cov = np.zeros(B, np.int32)
        full_t0 = W.t0_offsets(0, B, B)
        full_nz = W.noise_for(0, B, 7)
        for r in range(world):
            idx = W.shard_indices(B, world, r)
            cov[idx] += 1
            np.testing.assert_array_equal(W.t0_at(idx, B), full_t0[idx])
            np.testing.assert_array_equal(W.noise_at(idx, 7), full_nz[idx])
        assert np.all(cov == 1)


def test_round_robin_ranks_span_the_whole_figure8():
    """Every rank's robots cover the full period (same difficulty mix as one GPU): each
    rank has robots in every 1/64 of the period."""
    B, world = 65536 * 8, 8
    for r in range(world):
        t0 = W.t0_at(W.shard_indices(B, world, r), B)
        hist = np.histogram(t0, bins=64, range=(0, W.PERIOD))[0]
        assert hist.min() > 0.9 * hist.mean()


def test_rank_inputs_equal_global_slices():
    """Rank-local generation == slice of the single-process workload (no scatter needed)."""
    B, world = 3 * 65536 + 1000, 4
    full_t0 = W.t0_offsets(0, B, B)
    full_nz = W.noise_for(0, B, 7)
    for r in range(world):
        lo, hi = W.shard(B, world, r)
        np.testing.assert_array_equal(W.t0_offsets(lo, hi, B), full_t0[lo:hi])
        np.testing.assert_array_equal(W.noise_for(lo, hi, 7), full_nz[lo:hi])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B_total = 65536 * world
    idx = W.shard_indices(B_total, world, rank)
    lo, hi = int(idx[0]), int(idx[-1]) + 1
    counts = [idx.size - rank, rank, 0]                # fake per-rank status counts
    elapsed, tot = W.aggregate(dist, 0.5 + rank, counts, device="cpu")
    q.put((rank, lo, hi, elapsed, tot))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_two_ranks_aggregate():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=90) for _ in range(world))
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    B_total = 65536 * world
    assert [r[1] for r in res] == [0, 1] and res[-1][2] == B_total     # round-robin: r, r+W, ...
    for r in res:
        assert r[3] == 0.5 + (world - 1)                # slowest rank's time on every rank
        assert r[4] == [B_total - 1, 1, 0]              # status counts summed over ranks
