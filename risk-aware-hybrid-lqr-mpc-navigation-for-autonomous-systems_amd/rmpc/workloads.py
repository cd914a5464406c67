"""Synthetic BASELINE workloads and the batch split across ranks.

Robot i of a global batch of B robots follows the Figure-8 (A=2, a=0.5, dt=0.02) with time
offset t0_i = (i / B) * 2*pi/a (one full period over the batch) and starts at
x_ref(t0_i) + N(0, diag(.05^2, .05^2, .1^2)).  Noise is drawn per robot from a counter-based
generator keyed on (seed, i), so any subset of the batch is reproduced exactly by the rank
that owns it -- no data-path collective is needed to split the batch.

Robots are dealt to ranks round-robin (rank r owns i = r, r + W, r + 2W, ...), so every
rank's robots span the whole Figure-8 and every GPU gets the single-GPU difficulty mix.  A
contiguous split would hand the obstacle-adjacent arcs to a few ranks: at 8 GPUs, two ranks
would hold 17145 and 10754 robots beyond the lane-per-robot stage's cap against 0-46 on the
others (3552 at 1 GPU), and the slowest rank sets the job's time.
"""
import numpy as np

PERIOD = 2 * np.pi / 0.5

DEFAULT_OBS = [(1.0, 0.5, 0.2), (-0.5, -1.0, 0.25), (1.5, -0.3, 0.15)]     # run_simulation.py:215-219
UNION8_OBS = DEFAULT_OBS + [(-1.5, 0.5, 0.2), (0.0, 0.8, 0.15), (1.5, 0.8, 0.2),
                            (-0.8, -0.7, 0.15), (-0.3, -1.2, 0.15)]          # :191-212

CONFIGS = {
    # name: (horizon, obstacles, global batch at N=1, seed, what)
    "cfg2": dict(N=0, obs=[], B=4096, seed=0, what="LQR DARE+gain+apply, fp64"),
    "cfg3": dict(N=20, obs=DEFAULT_OBS, B=65536, seed=1, what="MPC QP N=20, 3 obstacles, fp64"),
    "cfg4": dict(N=30, obs=UNION8_OBS, B=32768, seed=2, what="MPC QP N=30, 8 obstacles"),
    "cfg5": dict(N=20, obs=DEFAULT_OBS, B=65536, seed=3, what="hybrid LQR/MPC step, N=20"),
}


# Performance settings of the contexts bench.py runs with batches in flight, per configuration
# (rmpc_ctx_set_stage_caps / _cold_start / _stage_passes / _side_stream; the QP optimum is the
# same under every setting).  tests/test_gpu_headline.py runs exactly these.  Measured choices:
# caps (9, 3) for config 3 (profiles/r05/session_46-48), (13, 4) LTI, (14, 6) config 4, (9, 4)
# config 5 (its MPC branch); zero-correction first sets in flight (session_27, _49); side
# streams off in flight (config 5's LQR branch too since round 6: ten in flight on 32 queues
# without them +8%, with them 20 streams oversubscribe the queues; profiles/r06);
# config 3's stage 1 in two passes, the first one PDAS solve long (profiles/r06: +2.6% at the
# driver's command over five pairs, +3% at 100 steps; configs 4 and LTI lose with passes);
# config 4's fp32 stage at one lane per robot in flight (profiles/r06: +13% in flight, three
# pairs; its one batch alone keeps the paired lanes, -20% otherwise).
INFLIGHT = {
    "cfg3": dict(caps=(9, 3), cold_start=1, passes=(1, 0), lanes=0, side=False),
    "lti": dict(caps=(13, 4), cold_start=1, passes=(0, 0), lanes=0, side=False),
    "cfg4": dict(caps=(14, 6), cold_start=1, passes=(0, 0), lanes=1, side=False),
    "cfg5": dict(caps=(9, 4), cold_start=1, passes=(0, 0), lanes=0, side=False),
}
# one batch at a time: the library's defaults
ALONE = dict(caps=(0, 0), cold_start=0, passes=(0, 0), lanes=0, side=True)


def inflight_settings(config, lti=False):
    """A copy of the in-flight settings of BASELINE config `config` (LTI: `solve()`)."""
    return dict(INFLIGHT["lti" if lti and config == "cfg3" else config])


def shard(B_total, world, rank):
    """Contiguous split [r*B/W, (r+1)*B/W) -- kept for tools; the bench uses shard_indices."""
    lo = (B_total * rank) // world
    hi = (B_total * (rank + 1)) // world
    return lo, hi


def shard_indices(B_total, world, rank):
    """Round-robin split: the global robot indices rank r owns (r, r + W, ...)."""
    return np.arange(rank, B_total, world, dtype=np.int64)


def t0_offsets(lo, hi, B_total):
    return (np.arange(lo, hi, dtype=np.float64) / B_total) * PERIOD


def t0_at(idx, B_total):
    """Time offsets of the robots with global indices idx."""
    return (np.asarray(idx, dtype=np.float64) / B_total) * PERIOD


def _noise_aligned(lo, hi, seed, sigma=(0.05, 0.05, 0.1)):
    """Per-robot N(0, sigma^2) keyed on (seed, global index); lo must be 65536-aligned."""
    out = np.empty((hi - lo, 3))
    for i0 in range(lo, hi, 65536):
        i1 = min(hi, i0 + 65536)
        ss = np.random.SeedSequence([seed, i0 // 65536])
        z = np.random.default_rng(ss).standard_normal((65536, 3))
        out[i0 - lo:i1 - lo] = z[: i1 - i0] * np.asarray(sigma)
    return out


def noise_for(lo, hi, seed, sigma=(0.05, 0.05, 0.1)):
    """Noise for an arbitrary [lo, hi) that may start inside a 65536-block."""
    b0 = (lo // 65536) * 65536
    full = _noise_aligned(b0, hi, seed, sigma)
    return full[lo - b0:]


def noise_at(idx, seed, sigma=(0.05, 0.05, 0.1)):
    """Noise of the robots with global indices idx (same values as noise_for)."""
    idx = np.asarray(idx, dtype=np.int64)
    if idx.size == 0:
        return np.empty((0, 3))
    lo, hi = int(idx.min()) // 65536 * 65536, int(idx.max()) + 1
    full = _noise_aligned(lo, hi, seed, sigma)
    return full[idx - lo]


def cfg5_t0(idx, A=2.0, a=0.5, obstacles=DEFAULT_OBS, d_mpc=0.7667):
    """BASELINE config 5 time offsets: even global indices on the arcs of the Figure-8 within
    d_mpc of an obstacle edge (the risk threshold 0.6 * risk >= 0.2 <=> d_edge <= 0.7667 m,
    risk_metrics.py:84-129 with run_simulation.py's weights), odd ones farther away, each
    pool swept in order over a 20000-point grid of one period -- about half the robots on the
    MPC branch (the start noise moves a few across)."""
    grid = np.linspace(0.0, PERIOD, 20000, endpoint=False)
    px, py = A * np.sin(a * grid), A * np.sin(a * grid) * np.cos(a * grid)   # reference_generator.py:86-101
    d = np.min([np.hypot(px - ox, py - oy) - r for ox, oy, r in obstacles], axis=0)
    near, far = grid[d <= d_mpc], grid[d > d_mpc]
    gi = np.asarray(idx, dtype=np.int64)
    return np.where(gi % 2 == 0, near[(gi // 2) % len(near)], far[(gi // 2) % len(far)])


def fleet_t0(idx, B_total, fleet=0, fleets=1):
    """Time offsets of fleet `fleet` of `fleets` independent fleets (bench.py's batches in
    flight): fleet f is the base workload shifted by f/fleets of the spacing between
    neighbouring robots, so no two fleets share a reference segment.  Fleet 0 is t0_at."""
    return (np.asarray(idx, dtype=np.float64) + fleet / max(1, fleets)) / B_total * PERIOD


def fleet_seed(seed, fleet=0):
    """Start-noise seed of fleet `fleet` (fleet 0: the config's own seed)."""
    return seed + 1000 * fleet


def broadcast_shared(dist, tensor, src=0):
    """SURVEY 8(e)'s setup collective: the shared read-only solve data (obstacles, weights)
    broadcast from rank `src` once before the rollout, so every rank solves against the same
    bits (in place; returns the tensor).  A no-op without a process group."""
    if dist is not None:
        dist.broadcast(tensor, src=src)
    return tensor


def gather_interleaved(dist, local, world, out=None):
    """SURVEY 8(e)'s batch gather: every rank's round-robin shard `local` ([B, ...], rank r
    holding global robots r, r + W, ...) all-gathered and interleaved back into global robot
    order ([W * B, ...]).  One all_gather_into_tensor (RCCL over xGMI on the GPU, gloo on the
    CPU) into `out` ([W * B, ...], allocated when None), then a transpose of its [W][B] view.
    Returns (global tensor, out)."""
    if out is None:
        out = local.new_empty((world * local.shape[0],) + tuple(local.shape[1:]))
    dist.all_gather_into_tensor(out, local.contiguous())
    g = out.view((world, local.shape[0]) + tuple(local.shape[1:])).transpose(0, 1)
    return g.reshape((-1,) + tuple(local.shape[1:])), out


def aggregate(dist, elapsed, counts, device="cpu"):
    """Cross-rank reduction of one bench run (the only collectives of the multi-GPU bench):
    the slowest rank's elapsed time (MAX) and the per-status robot counts (SUM).
    `dist` is torch.distributed (or None for a single process); tensors live on `device`
    (cuda for the RCCL backend, cpu for gloo)."""
    if dist is None:
        return float(elapsed), [int(c) for c in counts]
    import torch
    tt = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    if not len(counts):
        return float(tt.item()), []
    cc = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=device)
    dist.all_reduce(cc)
    return float(tt.item()), [int(v) for v in cc.tolist()]


def difficulty_key(x0, xr, ur, obs, d_safe=0.3, dt=0.02):
    """Predicted PDAS iterations of each robot (a heuristic for grouping robots into waves):
    hinge rows the zero-correction rollout violates (the free response of the start error
    under the reference inputs) + 8 |heading error| + 2 |position error|."""
    x0, xr, ur = np.asarray(x0), np.asarray(xr), np.asarray(ur)
    N = ur.shape[1] if ur.shape[1] < xr.shape[1] else xr.shape[1] - 1
    px, py = xr[:, :N, 0], xr[:, :N, 1]
    th = np.unwrap(xr[:, :N, 2], axis=1)
    vr = np.where(np.abs(ur[:, :N, 0]) > 0.01, ur[:, :N, 0], 0.1)
    e = x0 - xr[:, 0]
    eth = np.abs((e[:, 2] + np.pi) % (2 * np.pi) - np.pi)
    e0, e1, e2 = e[:, 0].copy(), e[:, 1].copy(), (e[:, 2] + np.pi) % (2 * np.pi) - np.pi
    viol = np.zeros(len(x0))
    for k in range(N):
        if k > 0:
            for ox, oy, r in obs:
                dx, dy = px[:, k] - ox, py[:, k] - oy
                dist = np.maximum(np.hypot(dx, dy), 1e-12)
                viol += (d_safe + r - (dx * (px[:, k] + e0 - ox) + dy * (py[:, k] + e1 - oy)) / dist) > 0
        e0 = e0 - vr[:, k] * np.sin(th[:, k]) * dt * e2
        e1 = e1 + vr[:, k] * np.cos(th[:, k]) * dt * e2
    return viol + 8 * eth + 2 * np.hypot(e[:, 0], e[:, 1])


def block_sorted_order(key, blk=512):
    """Permutation that sorts each block of `blk` consecutive robots by key (ascending)."""
    B = len(key)
    return np.concatenate([s + np.argsort(key[s:s + blk], kind="stable") for s in range(0, B, blk)])
