"""Multi-rank logic of bench.py on the CPU (gloo, world_size 2): the batch split, the
per-rank synthetic inputs, the timing collectives (MAX of time, SUM of status counts) and the
split-solve-gather of SURVEY 8(e) with the C port standing in for the device solve."""
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


def test_fleets_in_flight_are_distinct_workloads():
    """bench.py's batches in flight are independent fleets: fleet 0 is the config's own
    workload; the others have their own reference offsets and start noise."""
    B = 65536
    idx = W.shard_indices(B, 1, 0)
    np.testing.assert_array_equal(W.fleet_t0(idx, B, 0, 3), W.t0_at(idx, B))
    assert W.fleet_seed(1, 0) == 1
    t = [W.fleet_t0(idx, B, f, 3) for f in range(3)]
    nz = [W.noise_at(idx, W.fleet_seed(1, f)) for f in range(3)]
    for f in range(1, 3):
        assert np.all(t[f] > t[f - 1]) and np.all(t[f] < t[0] + W.PERIOD / B)
        assert not np.any(nz[f] == nz[0])


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


def _solve_worker(rank, world, port, q):
    """One rank of the bench's multi-GPU path with the C port as the solver: its round-robin
    shard of a cfg3 batch, solved, then all-gathered and interleaved back into global order by
    the function bench.py calls after every timed step (rmpc.workloads.gather_interleaved)."""
    import torch
    import torch.distributed as dist
    from oracle import cpu, figure8
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B_total, N = 4096, 20
    idx = W.shard_indices(B_total, world, rank)
    xr, ur = figure8.offset_segments(2.0, 0.5, 0.02, W.t0_at(idx, B_total), N + 1)
    x0 = xr[:, 0] + W.noise_at(idx, 1)
    p = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    # the shared obstacles from rank 0 (bench.py's setup broadcast); rank 1 starts from zeros
    obs = torch.tensor(W.DEFAULT_OBS, dtype=torch.float64) if rank == 0 else torch.zeros(3, 3, dtype=torch.float64)
    W.broadcast_shared(dist, obs)
    assert obs.tolist() == [list(o) for o in W.DEFAULT_OBS]
    out = cpu.mpc_solve_batch(p, x0, xr, ur, obs.numpy(), step_count=np.full(idx.size, 10, np.int32))
    u0 = torch.from_numpy(out["u0"])
    # the bench's own gather (rmpc.workloads.gather_interleaved, called by bench.py per step)
    g, buf = W.gather_interleaved(dist, u0, world)
    assert buf.shape == (B_total, 2)
    assert torch.equal(g[rank::world], u0)
    q.put((rank, g.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_gloo_two_ranks_split_solve_gather_matches_single_process():
    """a 4096-robot cfg3 batch split round-robin over two ranks, each shard solved
    (the C port standing in for the device), u0 gathered in global robot order on every rank:
    bit-identical to one process solving the whole batch."""
    from oracle import cpu, figure8
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_solve_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=150) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    B_total, N = 4096, 20
    idx = np.arange(B_total)
    xr, ur = figure8.offset_segments(2.0, 0.5, 0.02, W.t0_at(idx, B_total), N + 1)
    x0 = xr[:, 0] + W.noise_at(idx, 1)
    p = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    ref = cpu.mpc_solve_batch(p, x0, xr, ur, W.DEFAULT_OBS, step_count=np.full(B_total, 10, np.int32))
    for _, u0_global in res:
        np.testing.assert_array_equal(u0_global, ref["u0"])


def _bench(args, env=None, timeout=240):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=e, cwd="/tmp",
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world,per_rank,S", [(2, 512, 1), (8, 256, 1), (2, 256, 3)])
def test_bench_launcher_spawns_ranks_and_gathers(tmp_path, world, per_rank, S):
    """`python bench.py --gpus N` with no launcher starts its own N ranks (bench.spawn_ranks:
    child processes with RANK / WORLD_SIZE / MASTER_*), here through the CPU self-test mode
    (gloo, the C port in place of the device solve; the same timing loop, aggregate and
    gather_interleaved as the GPU run).  Exactly one JSON line comes back, with n_gpus N and the
    gathered leg; the gathered u0 is bit-identical to one process solving the whole batch.
    N = 8 is the driver's scaling node (BASELINE config 4): the launcher, the
    timing collectives and the 8-way interleaved gather run at the real rank count.
    S = 3: three fleets in flight (--inflight 3, bench.py's slots): the gathered leg rotates the
    slots like the timed loop, visits every one, and each slot's gathered u0 equals one process
    solving that fleet."""
    import json
    from oracle import cpu, figure8
    out = tmp_path / "u0.npy"
    r = _bench(["--gpus", str(world), "--selftest", "--selftest-batch", str(per_rank), "--steps", str(max(2, S)),
                "--warmup", "1", "--selftest-out", str(out)] + (["--inflight", str(S)] if S > 1 else []),
               timeout=360)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["selftest"] is True
    assert line["value"] > 0 and line["value_with_gather"] > 0
    assert line["gather_slots_visited"] == list(range(S))
    assert line["gather"].startswith("gloo all_gather")
    B_total, N = world * per_rank, 20
    assert line["config"]["global_batch"] == B_total and line["solver"]["optimal"] == B_total * S
    g = np.load(out)
    assert g.shape == (S, B_total, 2)
    idx = np.arange(B_total)
    p = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    for f in range(S):
        xr, ur = figure8.offset_segments(2.0, 0.5, 0.02, W.fleet_t0(idx, B_total, f, S), N + 1)
        x0 = xr[:, 0] + W.noise_at(idx, W.fleet_seed(W.CONFIGS["cfg3"]["seed"], f))
        ref = cpu.mpc_solve_batch(p, x0, xr, ur, W.DEFAULT_OBS, step_count=np.full(B_total, 10, np.int32))
        np.testing.assert_array_equal(g[f], ref["u0"])


@pytest.mark.timeout(300)
def test_bench_launcher_fails_when_a_rank_fails():
    """A rank that dies (status 3 after joining the group, while its peer waits in a
    collective) ends the whole job: the parent terminates the other rank, prints no JSON line and
    exits non-zero, well before any collective timeout."""
    import time
    t = time.time()
    r = _bench(["--gpus", "2", "--selftest", "--selftest-batch", "64", "--steps", "1", "--warmup", "0",
                "--selftest-fail-rank", "1"])
    assert r.returncode != 0
    assert "rank 1 of 2 exited with status 3" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert time.time() - t < 120


def test_bench_world_size_must_match_gpus():
    """Under a launcher, WORLD_SIZE and --gpus must agree (a torchrun of 2 ranks with --gpus 1
    would otherwise report the wrong n_gpus)."""
    r = _bench(["--gpus", "1", "--selftest"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 1" in r.stderr
