#!/usr/bin/env python3
"""Benchmark: batched MPC QP solves/s on MI355X (BASELINE.json metric, config 3 by default).

One step = one batched solve_with_ltv (mpc_controller.py:345-522) of every robot the rank
owns, inputs already resident in HBM, all of the reference's outputs produced (u0, u_seq,
x_pred, cost, status, slack_used, iterations).  N>1: one process per GPU, the batch is
weak-scaled (65536 robots per GPU), robots are independent, so there is no data-path
collective -- only the timing barrier and a max-reduction of the elapsed time.

Prints ONE JSON line on rank 0 (see DESIGN.md "Measurement" for every field).
"""
import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd")
for _p in (ROOT, PKG_DIR):
    if _p not in sys.path:
        sys.path.insert(0, _p)

# Version of the JSON line's field meanings.  3 (round 4 on): value_one_batch_alone and
# roofline.kernel_avg_ms are the library-default-caps launch; the in-flight-caps launch moved to
# value_one_batch_alone_inflight_caps (before round 4 value_one_batch_alone was that launch).
SCHEMA = 3
FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector (= FP64 matrix) dense peak, SURVEY.md 8(d)
FP32_PEAK_TFLOPS = 157.3    # MI355X FP32 vector dense peak (MI355X_MICROARCH.md chip table)
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md chip table (spec)


def canonical_flops(N, n_obs, iters):
    """SURVEY.md 8(d) algorithmic flops per QP solve (condensed dense model):
    condense 8N^3 + 2 n_o N^2, factor (N n_u)^3/3 + n_o N (N n_u)^2, per iteration
    2 (N n_u)^2 + 4 n_o N * N n_u  (n_u = 2)."""
    nu = 2
    condense = 8 * N ** 3 + 2 * n_obs * N ** 2
    factor = (N * nu) ** 3 / 3 + n_obs * N * (N * nu) ** 2
    per_it = 2 * (N * nu) ** 2 + 4 * n_obs * N * N * nu
    return condense + factor + per_it * iters


def kernel_flops(N, n_obs, iters):
    """What the kernel actually executes per solve (flop count of rmpc_mpc.hip):
    setup ~N(10 + 15 n_o), each active-set iteration = one block Riccati pass
    ~N(73 + 4 n_o) + nb*164 (nb = N at block size 1), outputs ~30 N."""
    return N * (10 + 15 * n_obs) + iters * (N * (73 + 4 * n_obs) + N * 164) + 30 * N


def cpu_threads():
    """Host threads for the CPU baseline: the job's CPU share.  gpurun boxes export
    OMP_NUM_THREADS=16 for a one-GPU job (the machine has 256 hardware threads, shared by its
    8 GPUs' jobs); without it, every CPU this process may run on."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return env if env > 0 else len(os.sched_getaffinity(0))


def host_info():
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def latest_profile(name):
    """Newest committed profiles/r*/<name> (PMC passes of this workload), or None."""
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", name)))
    return (json.load(open(fs[-1])), os.path.relpath(fs[-1], ROOT)) if fs else (None, None)


def algorithmic_bytes(N, n_obs, n_out_rows=True):
    """HBM bytes per solve: inputs x0 + x_refs (N+1 rows) + u_refs (N+1 rows) + step count;
    outputs u0 + cost + status + slack + iters (+ u_seq and x_pred)."""
    inb = 8 * (3 + 3 * (N + 1) + 2 * (N + 1)) + 4
    outb = 8 * 2 + 8 + 4 + 1 + 4
    if n_out_rows:
        outb += 8 * (2 * N + 3 * (N + 1))
    return inb + outb


# ---- multi-rank plumbing: one process per GPU ----------------------------------

def rank_env(args):
    """(world, rank, local rank) of this process.  Under a launcher (torchrun, or spawn_ranks
    below) WORLD_SIZE is set and must equal --gpus; without one, --gpus 1 is the single
    process and --gpus N > 1 returns world None: the caller starts the N ranks itself."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            return None, 0, 0
        return 1, 0, 0
    world = int(env_world)
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU "
                         "with --gpus equal to the launcher's process count")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def spawn_ranks(n, argv, grace_s=30.0):
    """`python bench.py --gpus N` with no launcher: start N child processes of this script, one
    per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (127.0.0.1
    unless MASTER_ADDR is given).  This parent never imports torch or touches a GPU, and never
    execs: the children are new processes (subprocess.Popen).  Each child dies with the parent
    (PR_SET_PDEATHSIG).  If any child fails or is killed the others are terminated and the
    parent exits non-zero; otherwise it relays rank 0's one JSON line (checking n_gpus == N)."""
    import signal
    import socket
    import subprocess
    import tempfile

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        free_port = s.getsockname()[1]
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = os.environ.get("MASTER_PORT", str(free_port))

    def die_with_parent():                 # runs in the child between fork and exec
        import ctypes
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)   # PR_SET_PDEATHSIG

    out0 = tempfile.TemporaryFile(mode="w+")
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR=addr, MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=out0 if r == 0 else sys.stderr, preexec_fn=die_with_parent))

    def stop_all(*_):
        for q in procs:
            if q.poll() is None:
                q.terminate()
        t_end = time.time() + grace_s
        for q in procs:
            try:
                q.wait(max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                q.kill()
                q.wait()
    old = {sig: signal.signal(sig, lambda s_, f_: (stop_all(), sys.exit(128 + s_))) for sig in (signal.SIGTERM, signal.SIGINT)}
    failed = None
    while failed is None and any(q.poll() is None for q in procs):
        for r, q in enumerate(procs):
            if q.poll() not in (None, 0):
                failed = (r, q.returncode)
                break
        time.sleep(0.1)
    if failed is None:
        failed = next(((r, q.returncode) for r, q in enumerate(procs) if q.returncode != 0), None)
    if failed is not None:
        stop_all()
    for sig, h in old.items():
        signal.signal(sig, h)
    if failed is not None:
        print(f"bench.py: rank {failed[0]} of {n} exited with status {failed[1]}", file=sys.stderr)
        return failed[1] if failed[1] > 0 else 128 - failed[1]
    out0.seek(0)
    lines = [ln for ln in out0.read().splitlines() if ln.startswith("{")]
    if len(lines) != 1:
        print(f"bench.py: rank 0 printed {len(lines)} JSON lines, expected 1", file=sys.stderr)
        return 1
    if json.loads(lines[0]).get("n_gpus") != n:
        print(f"bench.py: rank 0 reports n_gpus != {n}", file=sys.stderr)
        return 1
    print(lines[0], flush=True)
    return 0


def init_dist(args, world, local):
    """The process group of an N > 1 run: RCCL ("nccl", one GPU per rank, bound to cuda:local),
    or gloo for --rehearse-one-gpu / --selftest.  None for a single process."""
    if world == 1:
        return None
    import torch
    import torch.distributed as dist
    if args.selftest or args.rehearse_one_gpu:
        dist.init_process_group("gloo")
    else:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    return dist


def coll_device(args, dev):
    """Where collective tensors live: the rank's GPU for RCCL, the host for gloo."""
    import torch
    return torch.device("cpu") if (args.selftest or args.rehearse_one_gpu) else dev


def parallelism(args, world):
    s = f"batch-split x{world} (no data-path collective)"
    if args.rehearse_one_gpu and world > 1:
        s += "; rehearsal: every rank on cuda:0, gloo collectives (not a scaling number)"
    return s


def alone_times(run_one, stream, K, skip=2):
    """One batch at a time on one stream: (ms per launch for K launches back to back between two
    HIP events -- a single fleet's rate, the roofline's launch time -- and the mean ms of K more
    launches each between its own pair of events, whose packets sit between the launches)."""
    import numpy as np
    import torch
    for _ in range(skip):
        run_one()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(K):
        run_one()
    b.record(stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for e0, e1 in ev:
        e0.record(stream)
        run_one()
        e1.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / K, float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev]))


def timed_loop(step, steps, warmup, dist, sync, S=1):
    """The timing contract: max(W, S) untimed steps, then exactly K steps (step k on in-flight
    slot k mod S) bracketed by barrier + synchronize on both sides.  Returns this rank's
    elapsed seconds (the caller takes the MAX over ranks)."""
    sync()
    for k in range(max(warmup, S)):
        step(k)
    sync()
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    sync()
    if dist:
        dist.barrier()
    return time.perf_counter() - t0


def gather_loop(step, local_u0, dist, world, rank, steps, sync, cdev, S=1, stream_of=None):
    """N > 1: K more steps with SURVEY 8(e)'s batch gather inside the timed region, in the same
    pipeline as the timed loop: step k runs on in-flight slot i = k mod S, and right after its
    solve, slot i's u0 shard is all-gathered and interleaved back into global robot order
    (rmpc.workloads.gather_interleaved) on slot i's own stream (`stream_of(i)`), into a buffer
    of that slot's own -- so the collective waits only for its own batch and the other slots'
    batches stay in flight (RCCL over xGMI; gloo through the host).  Returns (slowest rank's
    elapsed s, the last gathered u0 [world * B, 2] of every slot on cdev, the slots visited)."""
    import contextlib
    import torch
    from rmpc import workloads as W
    bufs, last, visited = [None] * S, [None] * S, set()

    def step_gather(k):
        i = k % S
        step(k)
        with (torch.cuda.stream(stream_of(i)) if stream_of else contextlib.nullcontext()):
            last[i], bufs[i] = W.gather_interleaved(dist, local_u0(i).to(cdev), world, bufs[i])
        visited.add(i)
    for k in range(S):
        step_gather(k)
    sync()
    dist.barrier()
    sync()
    t = time.perf_counter()
    for k in range(steps):
        step_gather(k)
    sync()
    dist.barrier()
    elapsed = time.perf_counter() - t
    for i in range(S):
        assert bool((last[i][rank::world] == local_u0(i).to(cdev)).all()), i
    elapsed, _ = W.aggregate(dist, elapsed, [], device=cdev)
    return elapsed, last, sorted(visited)


def gather_label(dist, B, S):
    """What `value_with_gather` measures, named after the backend actually used."""
    be = dist.get_backend()
    coll = "RCCL all_gather over xGMI" if be == "nccl" else f"{be} all_gather through the host"
    return (f"{coll} of u0 ({B} x 2 fp64 per rank) after every step, on that step's in-flight slot's stream "
            f"(S = {S} slots, rotated as in the timed loop), inside the timed region")


def selftest_rank(args, world, rank):
    """--selftest: one rank of the multi-rank flow on the CPU (gloo), with the oracle's C port
    standing in for the device solve (a checker of the launcher and collectives, never a
    measurement): its round-robin shard of S config-3 fleets (--inflight S, bench.py's fleets),
    the setup broadcast, the timed loop over the slots, the gathered leg (every slot's u0
    gathered after its step) and the MAX / SUM aggregation -- the same functions as the GPU run.
    Rank 0 prints one JSON line (and saves the gathered u0 of every slot, [S, W * B, 2], with
    --selftest-out)."""
    import numpy as np
    import torch
    from oracle import cpu, figure8
    from rmpc import workloads as W

    dist = init_dist(args, world, 0)
    if rank == args.selftest_fail_rank:
        sys.exit(3)                        # the others now block in their first collective
    cfg = W.CONFIGS["cfg3"]
    S = max(1, args.inflight) if args.inflight_given else 1
    N, B_total = cfg["N"], args.selftest_batch * world
    idx = W.shard_indices(B_total, world, rank)
    fleets = []
    for f in range(S):
        xr, ur = figure8.offset_segments(2.0, 0.5, 0.02, W.fleet_t0(idx, B_total, f, S), N + 1)
        fleets.append((xr[:, 0] + W.noise_at(idx, W.fleet_seed(cfg["seed"], f)), xr, ur))
    obs = torch.tensor(cfg["obs"], dtype=torch.float64) if rank == 0 else torch.zeros(len(cfg["obs"]), 3, dtype=torch.float64)
    obs = W.broadcast_shared(dist, obs)
    p = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    res = [None] * S

    def step(k=0):
        x0, xr, ur = fleets[k % S]
        res[k % S] = cpu.mpc_solve_batch(p, x0, xr, ur, obs.numpy(), step_count=np.full(idx.size, 10, np.int32))
    nosync = lambda: None                                      # noqa: E731
    elapsed = timed_loop(step, args.steps, args.warmup, dist, nosync, S)
    u0 = lambda i: torch.from_numpy(res[i]["u0"])              # noqa: E731
    visited = [0]
    if dist is None:
        elapsed_g, g = None, [u0(i) for i in range(S)]
    else:
        elapsed_g, g, visited = gather_loop(step, u0, dist, world, rank, args.steps, nosync, torch.device("cpu"), S)
    st = np.concatenate([r["status"] for r in res])
    elapsed, counts = W.aggregate(dist, elapsed, [int((st == c).sum()) for c in (0, 1, 2)])
    line = {"metric": "SELFTEST (C port on the CPU, not a measurement): MPC QP solves/sec", "selftest": True,
            "value": B_total * args.steps / elapsed, "unit": "solves/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"cfg3 shape, {args.selftest_batch} robots/rank", "global_batch": B_total,
                       "parallelism": f"batch-split x{world}, gloo", "batches_in_flight": S},
            "solver": dict(optimal=counts[0], inaccurate=counts[1], fallback=counts[2])}
    if elapsed_g is not None:
        line["value_with_gather"] = B_total * args.steps / elapsed_g
        line["gather"] = gather_label(dist, idx.size, S)
        line["gather_slots_visited"] = visited
    if rank == 0:
        if args.selftest_out:
            np.save(args.selftest_out, torch.stack(g).numpy())
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (100 timed steps: with batches in flight the first and last few are not overlapped, so a
    # short run understates the steady state -- 20 steps read ~7% lower at config 3)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="cfg3", choices=["cfg2", "cfg3", "cfg4", "cfg5"],
                    help="BASELINE config (cfg3 = the metric's configuration, the default)")
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-pointer (PCIe-inclusive) timing")
    ap.add_argument("--f32", action="store_true", help="fp32 arithmetic for cfg3 too (A/B)")
    ap.add_argument("--f64", action="store_true", help="fp64 arithmetic for cfg4 (A/B against its fp32 pipeline)")
    ap.add_argument("--lti", action="store_true",
                    help="MPCController.solve (absolute-state LTI, mpc_node's path) instead of solve_with_ltv")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-closed-loop", action="store_true", help="skip the closed-loop (cold / warm) rates")
    ap.add_argument("--no-drop-in", action="store_true", help="skip the single-robot drop-in latency")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline work budget")
    ap.add_argument("--stage-caps", default=None,
                    help="FAST,TAIL: the in-flight contexts' stage caps instead of the tuned ones (sweeps)")
    ap.add_argument("--stage-passes", default=None,
                    help="C1[,C2]: the in-flight contexts' stage-1 passes (rmpc_ctx_set_stage_passes) "
                         "instead of the tuned ones; 0 = one pass")
    ap.add_argument("--presort", type=int, default=0,
                    help="A/B: order each fleet's robots by predicted difficulty within blocks of this size")
    ap.add_argument("--alone-side", type=int, default=None, choices=[0, 1],
                    help="config 5's one-batch-alone measurement: the context's side stream on (1, the "
                         "library default) or off (0).  Default: off when --hw-queues raised the queue "
                         "count (with 16 queues mapped, the side stream's fork/join per step costs more "
                         "than it overlaps: 108M against 146M steps/s; on HIP's default 4 queues the "
                         "side stream gives 171M)")
    ap.add_argument("--inflight-side", type=int, default=None, choices=[0, 1],
                    help="the in-flight contexts' side streams (A/B; default rmpc.workloads.INFLIGHT: off, "
                         "config 5 on)")
    ap.add_argument("--inflight", type=int, default=None,
                    help="batches in flight at once, each on its own stream with its own solver "
                         "context and outputs (step k runs on stream k mod S); default 8; configs 3 "
                         "(solve_with_ltv) and 5: 10 on 32 hardware queues (profiles/r06: config 3 "
                         "+1.9%% at 20 steps and +3.7%% at 100 over 8 on 16, config 5 +8%% without its "
                         "side streams); config 2 3 (its ~7 us LQR launches are host-bound: 758M "
                         "controls/s at 3 against 380M at 8)")
    ap.add_argument("--cold-start", type=int, default=1, choices=[0, 1],
                    help="in-flight contexts' first active sets (rmpc_ctx_set_cold_start): 1 zero-correction rows")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="hardware queues per process (GPU_MAX_HW_QUEUES, at most 32; HIP's default is 4): "
                         "each batch in flight needs a queue of its own, or two fleets' streams share one "
                         "in-order queue (0: leave the environment's setting); default 16, configs 3 "
                         "(solve_with_ltv) and 5: 32")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N>1 on a one-GPU box: every rank on cuda:0, gloo collectives through host "
                         "tensors (exercises the multi-rank bench flow; not a scaling number)")
    ap.add_argument("--selftest", action="store_true",
                    help="CPU-only self-test of the multi-rank flow (gloo, the C port in place of the "
                         "device solve): launcher, timing collectives and the batch gather")
    ap.add_argument("--selftest-batch", type=int, default=1024, help="--selftest: robots per rank")
    ap.add_argument("--selftest-out", default=None, help="--selftest: rank 0 saves the gathered u0 here (.npy)")
    ap.add_argument("--selftest-fail-rank", type=int, default=-1,
                    help="--selftest: this rank exits with status 3 after joining the group (launcher test)")
    args = ap.parse_args()
    args.inflight_given = args.inflight is not None
    ten = (args.config == "cfg3" and not args.lti) or args.config == "cfg5"     # 10 in flight on 32 queues
    if args.inflight is None:
        args.inflight = 3 if args.config == "cfg2" else (10 if ten else 8)
    if args.hw_queues is None:
        args.hw_queues = 32 if ten else 16
    if args.alone_side is None:
        args.alone_side = 0 if args.hw_queues > 4 else 1
    # (before anything initialises HIP: the setting is read once per process; spawned ranks
    # inherit it)
    if args.hw_queues > 0:
        cur = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(cur, args.hw_queues)))

    world, rank, local = rank_env(args)
    if world is None:                     # --gpus N > 1 without a launcher: start the N ranks
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if args.selftest:
        return selftest_rank(args, world, rank)
    # config 2's SciPy leg forks its worker pool, so it runs before the GPU is initialised
    pre = None
    if args.config == "cfg2" and world == 1 and not args.no_cpu_baseline:
        pre = cfg2_scipy_baseline(4096, args.cpu_seconds * 0.5)
    import numpy as np
    import torch

    if args.rehearse_one_gpu:
        local = 0
    torch.cuda.set_device(local)
    dist = init_dist(args, world, local)

    import rmpc
    from rmpc import workloads as W

    if args.config in ("cfg2", "cfg5"):
        return bench_other(args, world, rank, local, dist, pre)
    cfg = W.CONFIGS[args.config]
    N, obs_list, seed = cfg["N"], cfg["obs"], cfg["seed"]
    B_per = cfg["B"] if args.config == "cfg3" else 32768
    B_total = B_per * world
    idx = W.shard_indices(B_total, world, rank)        # round-robin: same difficulty mix per rank
    B = idx.size

    # ---- synthetic inputs (Figure-8 offsets + seeded noise), generated by the device
    # reference kernel and then made resident in HBM before anything is timed.  Each batch in
    # flight is its own fleet (rmpc.workloads.fleet_t0 / fleet_seed: other reference offsets,
    # other start noise): one fleet's closed loop cannot overlap its own steps, so the batches
    # in flight stand for independent fleets sharing the GPU, not copies of one batch.
    S = max(1, args.inflight)
    dev = torch.device(f"cuda:{local}")
    fleets = []
    for f in range(S):
        xr_f, ur_f = rmpc.batch.figure8_batch(W.fleet_t0(idx, B_total, f, S), N + 1, device=local)
        x0_f = xr_f[:, 0] + W.noise_at(idx, W.fleet_seed(seed, f))
        if args.presort:
            o = W.block_sorted_order(W.difficulty_key(x0_f, xr_f, ur_f, obs_list), args.presort)
            xr_f, ur_f, x0_f = xr_f[o], ur_f[o], x0_f[o]
        fleets.append(dict(x0_h=x0_f, xr_h=xr_f, ur_h=ur_f, x0=torch.from_numpy(x0_f).to(dev),
                           xr=torch.from_numpy(xr_f).to(dev), ur=torch.from_numpy(ur_f).to(dev)))
    x0_h, xr_h, ur_h = fleets[0]["x0_h"], fleets[0]["xr_h"], fleets[0]["ur_h"]
    x0, xr, ur = fleets[0]["x0"], fleets[0]["xr"], fleets[0]["ur"]
    obs = torch.tensor(obs_list, dtype=torch.float64, device=dev).reshape(-1, 3)
    cdev = coll_device(args, dev)          # collectives: the GPU (RCCL) or, for gloo, the host
    obs = W.broadcast_shared(dist, obs.to(cdev)).to(dev)   # rank 0's obstacles on every rank (setup, untimed)

    def new_out():
        return dict(u0=torch.empty(B, 2, dtype=torch.float64, device=dev),
                    u_seq=torch.empty(B, N, 2, dtype=torch.float64, device=dev),
                    x_pred=torch.empty(B, N + 1, 3, dtype=torch.float64, device=dev),
                    cost=torch.empty(B, dtype=torch.float64, device=dev),
                    status=torch.empty(B, dtype=torch.int32, device=dev),
                    slack_used=torch.empty(B, dtype=torch.uint8, device=dev),
                    iters=torch.empty(B, dtype=torch.int32, device=dev))
    # one output set, step counter, stream and solver context (rmpc slot) per batch in flight
    outs = [new_out() for _ in range(S)]
    out = outs[0]
    counts_sc = [torch.full((B,), 10, dtype=torch.int32, device=dev) for _ in range(S)]   # past the cold-start ramp
    step_count = counts_sc[0]
    # config 4 is specified in fp32 arithmetic (BASELINE.json); config 3 in fp64
    f32 = (args.config == "cfg4" and not args.f64) or args.f32
    p = rmpc._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0,
                                0.02, block_size=1, ltv=not args.lti, precision=1 if f32 else 0)
    stream = torch.cuda.current_stream()
    alone_default_s = None
    streams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(S - 1)]
    # with batches in flight the chip's idle time is filled by the other batches, and a longer
    # lane-per-robot stage (less work for the lane-group tail) pays; the zero-correction first
    # sets lower the total PDAS work; side streams would add to the streams sharing the
    # hardware queues (rmpc.workloads.INFLIGHT: the settings, and where each was measured)
    cset = W.inflight_settings(args.config, args.lti) if S > 1 else dict(W.ALONE)
    if args.stage_caps:
        cset["caps"] = tuple(int(v) for v in args.stage_caps.split(","))
    if args.stage_passes:
        cset["passes"] = tuple(int(v) for v in (args.stage_passes + ",0").split(",")[:2])
    if S > 1:
        cset["cold_start"] = args.cold_start
        if args.inflight_side is not None:
            cset["side"] = bool(args.inflight_side)
    caps = cset["caps"]
    for i in range(S):
        rmpc.batch.configure(cset, device=local, slot=i)

    def step(k=0):
        i = k % S
        fl = fleets[i]
        rmpc.batch.mpc_solve_batch_dev(p, fl["x0"], fl["xr"], fl["ur"], obs, outs[i], step_count=counts_sc[i],
                                       device=local, stream=streams[i], slot=i)

    # inputs, outputs and step counters were written on the default stream: the other
    # streams start only after that work (they are non-blocking streams)
    elapsed = timed_loop(step, args.steps, args.warmup, dist, torch.cuda.synchronize, S)
    # one batch's launches on their own (nothing else in flight; HIP events on the launch
    # stream): the roofline's launch time
    k_ms, k_evt_ms = alone_times(lambda: step(0), stream, args.steps)
    k_avg_s = k_ms / 1e3
    # ... and with the library's default stage caps on a context of its own (what one batch at
    # a time would use; its side stream on, rmpc_ctx_set_side_stream)
    if S > 1:
        rmpc.batch.configure(W.ALONE, device=local, slot=S)
        alone_default_s = alone_times(lambda: rmpc.batch.mpc_solve_batch_dev(
            p, x0, xr, ur, obs, outs[0], step_count=counts_sc[0], device=local, stream=stream, slot=S),
            stream, args.steps)[0] / 1e3
    if alone_default_s is None:
        alone_default_s = k_avg_s

    # the roofline prices one batch alone at the library's defaults: the launch the rocprofv3
    # one-batch statistics and the PMC passes (bench.py --inflight 1) see
    k_roof_s = alone_default_s
    # per-stage device time of that launch (separate, untimed pass: events between the
    # pipeline's kernels; only the lane-per-robot pipeline has stages)
    rmpc.batch.configure(dict(W.ALONE, side=cset["side"]), device=local, slot=0)
    rmpc.batch.set_stage_timing(True, device=local)
    stage = []
    try:
        for _ in range(max(3, min(args.steps, 10))):
            step()
            stage.append(rmpc.batch.mpc_stage_times(device=local))
        stage_ms = [float(v) for v in np.mean(np.asarray(stage), axis=0)]
    except rmpc.RmpcError:
        stage_ms = None
    rmpc.batch.set_stage_timing(False, device=local)
    rmpc.batch.configure(cset, device=local, slot=0)

    # N > 1: the same K steps again with the batch gather of u0 inside the timed region
    # (SURVEY 8(e)'s collective: RCCL all_gather over xGMI; the round-robin shards interleave
    # back into global robot order by a transpose of the [world][B] result)
    elapsed_g = None
    if dist:
        elapsed_g, _, gather_slots = gather_loop(step, lambda i: outs[i]["u0"], dist, world, rank, args.steps,
                                                 torch.cuda.synchronize, cdev, S, lambda i: streams[i])

    st = out["status"].cpu().numpy()
    its = out["iters"].cpu().numpy()
    counts = [int((st == 0).sum()), int((st == 1).sum()), int((st == 2).sum())]
    # the only collectives: MAX of the elapsed time, SUM of the status counts
    elapsed, counts = W.aggregate(dist, elapsed, counts, device=cdev)
    stats = dict(optimal=counts[0], inaccurate=counts[1], fallback=counts[2],
                 iters_mean=round(float(its.mean()), 3),
                 iters_p99=float(np.percentile(its, 99)), iters_max=int(its.max()),
                 slack_active_frac=round(float(out["slack_used"].float().mean().item()), 4))

    n_obs = len(obs_list)
    fast_name = "mpc_ltv_fast_kernel"
    tail_name = "mpc_group_kernel"
    pipe = "fp64 VALU lane-per-robot stage + lane-group VALU Riccati tail (MFMA unused)"
    if f32:
        pipe = pipe.replace("fp64 VALU lane-per-robot stage",
                            "fp32 VALU lane-per-robot stage (active sets) + fp64 refinement pass of the same kernel")
    # config 4's fp32 stage is priced at the FP32 vector peak (its fp64 tail is a minority)
    peak = FP32_PEAK_TFLOPS if f32 else FP64_PEAK_TFLOPS
    flops = canonical_flops(N, n_obs, float(its.mean()))
    kflops = kernel_flops(N, n_obs, float(its.mean()))
    abytes = algorithmic_bytes(N, n_obs)
    achieved = flops * B / k_roof_s / 1e12
    line = {
        "metric": "MPC QP solves/sec (N=20, nx=3, nu=2) at 1/2/4/8 MI355X; max |u-u_ref|",
        "value": B_total * args.steps / elapsed,
        # the same batch with nothing else in flight (launches back to back between two HIP
        # events): with the library's defaults, what one batch at a time runs (the roofline's
        # launch), and with the in-flight stage caps
        "value_one_batch_alone": B_total / alone_default_s,
        "value_one_batch_alone_inflight_caps": B_total / k_avg_s,
        "schema": SCHEMA,
        "unit": "solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32+f64" if f32 else "f64",     # config 4: fp32 active-set pass, fp64 refinement
        "data": "synthetic: Figure-8 references at per-robot time offsets + seeded N(0,[.05,.05,.1]) "
                "start noise (SURVEY.md 8(d))",
        "config": {"workload": f"{args.config}: {'solve (LTI)' if args.lti else 'solve_with_ltv'}, N={N}, {n_obs} obstacles, "
                               f"Q=[15,15,50] R=[.1,.1] P=[30,30,40] rho=5000, {B_per} robots/GPU",
                   "robots_per_gpu": B_per, "global_batch": B_total, "horizon": N,
                   "n_obstacles": n_obs, "parallelism": parallelism(args, world),
                   "batches_in_flight": S, "stage_caps": list(caps) if caps[0] else "library default",
                   "stage_passes": list(cset["passes"]) if cset["passes"][0] else "one pass",
                   "zero_correction_first_sets": bool(cset["cold_start"])},
        # compute-bound path on the vector ALU (MFMA unused by the default pipeline): priced at
        # the FP64 (FP32 for config 4) vector peak.  `achieved`/`frac` use SURVEY 8(d)'s
        # canonical condensed-QP flop count; `frac_executed` is what the kernels actually
        # execute (PMC fp64 VALU op counters, profiles/r*/pmc_flops.json)
        "roofline": {"bound": "valu-fp32" if f32 else "valu-fp64", "achieved": achieved, "peak": peak,
                     "unit": "TFLOP/s", "frac": achieved / peak, "traffic": None,
                     "pipe": pipe,
                     "kernel": f"MPC launch: {fast_name} -> {tail_name} -> mpc_solve_kernel",
                     "kernel_avg_ms": k_roof_s * 1e3,
                     "kernel_avg_ms_note": "one batch alone at the library's default stage caps (value_one_batch_alone): K launches back to back on one stream between two HIP events",
                     "inflight_caps_launch_ms": k_avg_s * 1e3,
                     "inflight_caps_launch_ms_own_events": k_evt_ms,
                     "stage_ms": None if stage_ms is None else {
                         fast_name: stage_ms[0], tail_name: stage_ms[1],
                         "mpc_solve_kernel": stage_ms[2]},
                     "flops_per_solve_canonical": flops,
                     "flops_per_solve_executed": kflops,
                     "executed_tflops": kflops * B / k_roof_s / 1e12,
                     "algorithmic_bytes_per_solve": abytes,
                     "hbm_gbs_algorithmic": abytes * B / k_roof_s / 1e9,
                     "hbm_frac": abytes * B / k_roof_s / 1e9 / HBM_PEAK_GBS,
                     # kernel_avg_ms / achieved / frac: one batch's launch alone (library
                     # defaults, nothing else in flight); the job's own rate with S batches in flight:
                     "achieved_in_flight": flops * B_total * args.steps / elapsed / world / 1e12,
                     "frac_in_flight": flops * B_total * args.steps / elapsed / world / 1e12 / peak,
                     "frac_in_flight_note": "canonical flop model (SURVEY 8(d), ~2.1e5 flops per solve) at the "
                                            "in-flight rate: near 1 it is the model that saturates, not the "
                                            "hardware (the kernels execute ~4e4); frac_executed_in_flight "
                                            "(PMC) is the hardware figure"},
        "solver": stats,
    }
    if elapsed_g is not None:
        line["value_with_gather"] = B_total * args.steps / elapsed_g
        line["gather"] = gather_label(dist, B, S)
        line["gather_slots_visited"] = gather_slots

    # ---- PCIe-inclusive rate (rank 0, N=1 only; never `value`): the host-pointer C-ABI
    # (rmpc_mpc_solve_batch) with pageable numpy buffers, staged H2D/D2H by the library
    if world == 1 and rank == 0 and not args.no_pcie:
        pc = {}
        for tag, seq in (("full_outputs", True), ("u0_only", False)):
            sc_h = np.full(B, 10, np.int32)
            rmpc.batch.mpc_solve_batch(p, x0_h, xr_h, ur_h, obs_list, step_count=sc_h,
                                       device=local, want_seq=seq)
            ts = []
            for _ in range(5):
                t = time.perf_counter()
                rmpc.batch.mpc_solve_batch(p, x0_h, xr_h, ur_h, obs_list, step_count=sc_h,
                                           device=local, want_seq=seq)
                ts.append(time.perf_counter() - t)
            t_med = float(np.median(ts))
            pc[tag] = {"value": B / t_med, "ms_per_call": t_med * 1e3}
        pc["unit"] = "solves/s"
        pc["note"] = ("host numpy in/out through the host-pointer C-ABI, median of 5 calls; "
                      "full_outputs also returns u_seq and x_pred")
        line["pcie_inclusive"] = pc

    # ---- closed loop (rank 0, N=1, config 3 only; never `value`): run_simulation.py's MPC loop
    # on the device, cold and with the warm start across calls (rmpc_ctx_set_warm_start)
    if world == 1 and rank == 0 and args.config in ("cfg3", "cfg4") and not args.lti and not args.no_closed_loop:
        line["closed_loop"] = closed_loop(dev, B, obs_list, N, f32)

    # ---- single-robot drop-in latency (rank 0, N=1, config 3 runs only; never `value`)
    seqs = None
    if world == 1 and rank == 0 and args.config == "cfg3" and not args.lti and not args.no_drop_in:
        line["drop_in_latency"], seqs = drop_in_latency(local)

    # ---- CPU baseline (rank 0, N=1 only): the oracle's C restatement of the same algorithm
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        from oracle import cpu
        threads = cpu_threads()
        cp = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
        # the device pipeline's stage caps (rmpc_api.cpp), so the port follows the same iterate
        # path: fast PDAS cap 7 (LTI 9, N = 30: 12), then 4 (N = 30: 6) tail PDAS solves
        caps = (9, 4) if args.lti else ((7, 4) if N <= 20 else (12, 6))
        cpu.set_pdas_caps(*caps)
        nsamp = min(B, 16384)
        sl = slice(0, B, B // nsamp)       # strided: covers the whole Figure-8 period
        sc = np.full(nsamp, 10, np.int32)
        cpu.mpc_solve_batch(cp, x0_h[sl], xr_h[sl], ur_h[sl], obs_list, step_count=sc.copy(),
                            threads=threads)   # warm
        reps, t_cpu, res = 0, 0.0, None
        while t_cpu < args.cpu_seconds * 0.8 and reps < 1000:
            t = time.perf_counter()
            res = cpu.mpc_solve_batch(cp, x0_h[sl], xr_h[sl], ur_h[sl], obs_list,
                                      step_count=sc.copy(), threads=threads)
            t_cpu += time.perf_counter() - t
            reps += 1
        s1 = slice(0, B, B // 2048)
        n1 = len(range(*s1.indices(B)))
        t = time.perf_counter()
        cpu.mpc_solve_batch(cp, x0_h[s1], xr_h[s1], ur_h[s1], obs_list,
                            step_count=np.full(n1, 10, np.int32), threads=1)
        t1 = time.perf_counter() - t
        gpu_useq = out["u_seq"].cpu().numpy()[sl]
        both = (res["status"] == 0) & (st[sl] == 0)
        du = float(np.abs(gpu_useq[both] - res["u_seq"][both]).max())
        # every fleet in flight against the port on a strided 4096-robot sample of its own
        # inputs (the last timed step of its slot): u_seq and x_pred
        du_fleet = []
        for f in range(S):
            fl, of = fleets[f], outs[f]
            s4 = slice(0, B, max(1, B // 4096))
            rf = cpu.mpc_solve_batch(cp, fl["x0_h"][s4], fl["xr_h"][s4], fl["ur_h"][s4], obs_list,
                                     step_count=np.full(len(range(*s4.indices(B))), 10, np.int32),
                                     threads=threads)
            ok = (rf["status"] == 0) & (of["status"].cpu().numpy()[s4] == 0)
            du_fleet.append({
                "u_seq": float(np.abs(of["u_seq"].cpu().numpy()[s4][ok] - rf["u_seq"][ok]).max()),
                "x_pred": float(np.abs(of["x_pred"].cpu().numpy()[s4][ok] - rf["x_pred"][ok]).max()),
                "optimal_both": int(ok.sum())})
        cpu.set_pdas_caps(0, 0)
        line["cpu_baseline"] = {
            "value": nsamp * reps / t_cpu, "unit": "solves/s", "cores": threads, "kind": "port",
            "sample": f"{nsamp} robots (every {B // nsamp}th) of the same workload x {reps} reps "
                      f"(oracle/c/rmpc_cpu.c, OpenMP, same algorithm, stage caps {caps} and outputs)",
            "single_thread_solves_per_s": n1 / t1,
            # SURVEY 8(d) names OpenMP over all host cores; the job may use its share only (gpurun:
            # OMP_NUM_THREADS=16 of the machine's hardware threads, shared by 8 GPUs' jobs), so the
            # all-core figure is the measured per-thread rate scaled to every hardware thread --
            # a projection (perfect scaling, no SMT loss), never measured here
            "all_host_threads_projected": {"value": nsamp * reps / t_cpu / threads * (os.cpu_count() or threads),
                                           "threads": os.cpu_count(), "kind": "projection from the measured rate"},
            "reference_published_ms_per_solve": 82.6,
            "reference_published_note": "CVXPY/OSQP N=6 logged mean, hardware unstated (BASELINE.md)",
            "host": host_info()}
        if f32:
            line["cpu_baseline"]["note"] = ("the C port computes in fp64; the GPU path finds the active sets in fp32 "
                                            "and re-solves / re-certifies them in fp64 (outputs fp64-exact)")
        line["max_abs_du_vs_cpu_port"] = du
        line["max_abs_diff_vs_cpu_port_per_fleet"] = du_fleet
        if seqs:
            # the C port, one thread, one robot per call, on the drop-in loop's own inputs
            for (Nd, bs), (xs, xrs, urs) in seqs.items():
                cpd = cpu.mpc_params(Nd, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02,
                                     block_size=bs)
                sc1 = np.full(1, 10, np.int32)
                ts = []
                for k in range(len(xs)):
                    t = time.perf_counter()
                    cpu.mpc_solve_batch(cpd, xs[k:k + 1], xrs[k:k + 1], urs[k:k + 1], W.DEFAULT_OBS, step_count=sc1,
                                        threads=1)
                    ts.append(time.perf_counter() - t)
                line["drop_in_latency"][f"N{Nd}_bs{bs}"]["cpu_port_1thread_median_us"] = float(np.median(ts[10:])) * 1e6
    # HBM traffic and executed flops per launch from the committed PMC passes of this workload
    # (rocprofv3 --pmc, separate passes; scripts/pmc_hbm.sh, scripts/pmc_flops.sh)
    if not args.lti and not args.f32 and not args.f64 and args.config in ("cfg3", "cfg4"):
        pmc_into_roofline(line["roofline"], "" if args.config == "cfg3" else "_" + args.config, abytes * B, k_roof_s,
                          args.steps / elapsed if S > 1 else None)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()




def pmc_into_roofline(roof, suffix, alg_bytes, k_avg_s, launches_per_s=None):
    """Fill roofline.traffic (HBM bytes per launch, PMC FETCH_SIZE + WRITE_SIZE with the gfx950
    corrections) and the executed-flops fraction from the newest committed profiles/r*/
    pmc_traffic<suffix>.json and pmc_flops<suffix>.json (this workload's own passes).
    frac_executed prices each precision at its own vector peak: (fp64 / FP64 peak + fp32 / FP32
    peak) / launch time."""
    tr, src = latest_profile(f"pmc_traffic{suffix}.json")
    if tr:
        roof["traffic"] = tr["traffic_bytes_per_launch"]
        roof["traffic_unit"] = f"bytes/launch (PMC, {src})"
        if alg_bytes:
            roof["traffic_vs_algorithmic"] = tr["traffic_bytes_per_launch"] / alg_bytes
    fl, src = latest_profile(f"pmc_flops{suffix}.json")
    if fl:
        e64, e32 = fl["fp64_flops_per_launch"], fl.get("fp32_flops_per_launch", 0.0)
        roof["executed_flops_per_launch"] = {"fp64": e64, "fp32": e32}
        roof["achieved_executed"] = (e64 + e32) / k_avg_s / 1e12
        roof["frac_executed"] = (e64 / FP64_PEAK_TFLOPS + e32 / FP32_PEAK_TFLOPS) / 1e12 / k_avg_s
        roof["executed_source"] = (f"{src}: 64 x (2 FMA + ADD + MUL + TRANS) VALU instructions per precision "
                                   "(full-wave count: an upper bound)")
    # the headline's own executed-flops fraction: the PMC op counters of the in-flight pipeline
    # (scripts/inflight_run.py: the bench's in-flight settings, every dispatch a batch of the
    # timed loop's kind) times the launches per second the timed loop achieved
    ti, src_t = latest_profile(f"pmc_traffic_inflight{suffix}.json")
    if ti and launches_per_s:
        roof["traffic_in_flight"] = ti["traffic_bytes_per_launch"]
        roof["traffic_in_flight_source"] = f"{src_t} (PMC, the in-flight settings; bytes per launch)"
        if alg_bytes:
            roof["traffic_in_flight_vs_algorithmic"] = ti["traffic_bytes_per_launch"] / alg_bytes
    fi, src = latest_profile(f"pmc_flops_inflight{suffix}.json")
    if fi and launches_per_s:
        e64, e32 = fi["fp64_flops_per_launch"], fi.get("fp32_flops_per_launch", 0.0)
        roof["executed_flops_per_launch_in_flight"] = {"fp64": e64, "fp32": e32}
        roof["achieved_executed_in_flight"] = (e64 + e32) * launches_per_s / 1e12
        roof["frac_executed_in_flight"] = (e64 / FP64_PEAK_TFLOPS + e32 / FP32_PEAK_TFLOPS) * launches_per_s / 1e12
        roof["executed_in_flight_source"] = (f"{src} (in-flight settings) x {launches_per_s:.4g} launches/s "
                                             "of the timed loop")


REF_LOGGED_SOLVE_MS = 82.6   # mean solve_time_ms of logs/controls_20260208_014109.csv


def drop_in_latency(local, n_calls=200, skip=10):
    """The reference's own performance figure is one robot's per-solve latency (solve_time_ms,
    mpc_controller.py:360, 482; 82.6 ms mean in logs/controls_20260208_014109.csv, CVXPY/OSQP,
    N = 6).  Here: rmpc.MPCController.solve_with_ltv for ONE robot through the host-array C-ABI
    (numpy in, numpy out, synchronous), the reference's controller settings, warm start on (the
    controller's own context, as the reference solves with warm_start=True), closed loop along
    the Figure-8 with the plant stepped between solves (untimed), at run_simulation.py's N = 6 /
    bs = 2 (:164-176) and at config 1's N = 20.  Wall clock per call, after `skip` calls.
    Returns the latencies and the (x0, x_refs, u_refs) sequence of each size."""
    import numpy as np
    import rmpc
    from rmpc import workloads as W
    res, seqs = {}, {}
    for N, bs in ((6, 2), (20, 1)):
        c = rmpc.MPCController(horizon=N, Q_diag=[15, 15, 50], R_diag=[.1, .1], P_diag=[30, 30, 40],
                               d_safe=0.3, slack_penalty=5000.0, v_max=2.0, omega_max=3.0, dt=0.02,
                               block_size=bs, device=local)
        xr_all, ur_all = rmpc.batch.figure8_batch(np.arange(n_calls) * 0.02, N + 1, device=local)
        x = xr_all[0, 0] + np.array([0.05, -0.05, 0.1])
        obs = [rmpc.Obstacle(*o) for o in W.DEFAULT_OBS]
        ts, rep, its, seq, nonopt = [], [], [], [], 0
        for k in range(n_calls):
            t = time.perf_counter()
            s = c.solve_with_ltv(x, xr_all[k], ur_all[k], obs)
            ts.append(time.perf_counter() - t)
            rep.append(s.solve_time_ms)
            its.append(s.iterations)
            seq.append(x.copy())
            nonopt += s.status != "optimal"
            x = rmpc.batch.plant_step_batch(x[None], s.optimal_control[None], 0.02, 2.0, 3.0, device=local)[0]
        us = np.asarray(ts[skip:]) * 1e6
        res[f"N{N}_bs{bs}"] = {"median_us": float(np.median(us)), "p90_us": float(np.percentile(us, 90)),
                               "solve_time_ms_median": float(np.median(rep[skip:])),
                               "iters_mean": float(np.mean(its[skip:])), "calls": n_calls - skip, "not_optimal": nonopt,
                               "vs_reference_logged_mean": REF_LOGGED_SOLVE_MS * 1e3 / float(np.median(us))}
        seqs[(N, bs)] = (np.asarray(seq), xr_all, ur_all)
    res["reference_logged_mean_ms"] = REF_LOGGED_SOLVE_MS
    res["note"] = ("one robot per call: MPCController.solve_with_ltv (host numpy in/out, 3 kernel launches, "
                   "synchronous), closed loop on the Figure-8 with 3 obstacles, warm start on; the reference's "
                   "82.6 ms is CVXPY/OSQP at N=6 on unstated hardware")
    return res, seqs


def closed_loop(dev, B, obs_list, N=20, f32=False, K=50, fleets_max=3, hybrid=False, t0=None):
    """run_simulation.py's MPC loop (mpc_rate 1: one solve_with_ltv per robot and control step,
    then the plant) for fleets of B robots on the device (rmpc_rollout_batch_dev), from seeded
    noisy starts over one Figure-8 period; 1 and `fleets_max` fleets at once (one context and
    stream each), each from a cold start and with the warm start across calls (the reference's
    warm_start=True / get_warm_start, mpc_controller.py:272-277, 524-538).  Median of 3 runs of
    K steps after one untimed run.  Returns solves/s and the warm/cold closed-loop difference."""
    import ctypes as C

    import numpy as np
    import torch

    import rmpc
    from rmpc import _native as nat
    from rmpc import workloads as W
    lib = nat.load()
    mp = nat.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02,
                        precision=1 if f32 else 0)
    idx = np.arange(B)
    obs = torch.tensor(obs_list, dtype=torch.float64, device=dev).reshape(-1, 3)
    p = lambda t: C.c_void_p(t.data_ptr())                      # noqa: E731
    fl = []
    lp = nat.lqr_params([15, 15, 8], [.1, .1], 0.02, 2.0, 3.0)
    kp = nat.risk_params()
    for f in range(fleets_max):
        if t0 is None:
            start = ((idx * 628 + f * 628 // fleets_max) // B % 628).astype(np.int32)   # one period: 628 rows
        else:                              # the config's own time offsets (config 5: near obstacles)
            start = ((np.rint(np.asarray(t0) / 0.02).astype(np.int64) + f) % 628).astype(np.int32)
        xr0, _ = rmpc.batch.figure8_batch(start * 0.02, 1)
        x0 = xr0[:, 0] + W.noise_at(idx, W.fleet_seed(1, f))
        fl.append(dict(start=torch.from_numpy(start).to(dev), x0=torch.from_numpy(x0).to(dev),
                       states=torch.empty(B, K + 1, 3, dtype=torch.float64, device=dev),
                       controls=torch.empty(B, K, 2, dtype=torch.float64, device=dev),
                       cnt=torch.zeros(4, dtype=torch.int64, device=dev),
                       stream=torch.cuda.Stream(device=dev), ctx=nat.context(dev.index or 0, 16 + f)))
    rp = nat.RolloutParams()
    rp.mode, rp.steps, rp.table_len, rp.mpc_rate, rp.plant_method = 2 if hybrid else 1, K, 1000, 1, 0
    rp.dt, rp.A, rp.a, rp.v_max, rp.omega_max = 0.02, 2.0, 0.5, 2.0, 3.0
    torch.cuda.synchronize()
    res, states = {}, {}
    for S in (1, fleets_max):
        for warm in (False, True):
            for f in fl[:S]:
                nat.check(lib.rmpc_ctx_set_warm_start(f["ctx"], int(warm)), "rmpc_ctx_set_warm_start")

            def run():
                for f in fl[:S]:
                    nat.check(lib.rmpc_rollout_batch_dev(f["ctx"], C.byref(rp), C.byref(lp) if hybrid else None,
                                                         C.byref(mp), C.byref(kp) if hybrid else None, B,
                                                         p(f["start"]), p(f["x0"]), p(obs), obs.shape[0],
                                                         p(f["states"]), p(f["controls"]), None, p(f["cnt"]),
                                                         C.c_void_p(f["stream"].cuda_stream)),
                              "rmpc_rollout_batch_dev")
            run()
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                t = time.perf_counter()
                run()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t)
            res[f"{'warm' if warm else 'cold'}_{S}_fleet{'s' if S > 1 else ''}"] = S * B * K / float(np.median(ts))
            states.setdefault(warm, fl[0]["states"].cpu().numpy())
            cnt = fl[0]["cnt"].cpu().numpy()
            assert cnt[1:].sum() == 0 and (hybrid or cnt[0] == B * K)   # every solve certified optimal
    for f in fl:
        nat.check(lib.rmpc_ctx_set_warm_start(f["ctx"], 0), "rmpc_ctx_set_warm_start")
    res.update({
        "unit": "solves/s",
        "workload": f"run_simulation.py {'hybrid' if hybrid else 'MPC'} loop on the device (rmpc_rollout_batch_dev, mpc_rate 1, the config's "
                    f"QP, N={N}, {obs.shape[0]} obstacles{', fp32 request' if f32 else ''}): {B} robots per fleet x "
                    f"{K} steps, seeded noisy starts over one Figure-8 period; fleets in flight on their own "
                    f"contexts and streams",
        "warm_start": "rmpc_ctx_set_warm_start: each solve starts from the robot's previous certified sets "
                      f"shifted one step, first-stage cap {4 if f32 else 2} (library default with warm sets)",
        "max_abs_state_diff_warm_vs_cold": float(np.abs(states[True] - states[False]).max())})
    return res


def _timed(args, step, dist, dev, S=1):
    """W warm-up steps, then K steps between barrier + synchronize, step k on in-flight slot
    k mod S; then one batch alone on the launch stream (alone_times).  Returns (elapsed s,
    (ms per launch back to back, ms per launch between its own events))."""
    import torch
    stream = torch.cuda.current_stream()
    elapsed = timed_loop(step, args.steps, args.warmup, dist, torch.cuda.synchronize, S)
    return elapsed, alone_times(lambda: step(0), stream, args.steps)


def _scipy_lqr_chunk(args):
    """SciPy leg of the config-2 CPU baseline (one worker): DARE + solve + control law per
    robot exactly as lqr_controller.py:116-132/191-215 call them, no gain cache."""
    x, xr, ur = args
    import numpy as np
    from scipy.linalg import solve_discrete_are
    from threadpoolctl import threadpool_limits
    threadpool_limits(1)                   # one BLAS thread per worker (no oversubscription)
    Q, R, dt = np.diag([15.0, 15.0, 8.0]), np.diag([0.1, 0.1]), 0.02
    t = time.perf_counter()
    for b in range(len(x)):
        v, th = ur[b, 0], xr[b, 2]
        if abs(v) < 1e-6:
            v = 0.01
        s_, c_ = np.sin(th), np.cos(th)
        A = np.array([[1.0, 0.0, -v * s_ * dt], [0.0, 1.0, v * c_ * dt], [0.0, 0.0, 1.0]])
        Bm = np.array([[c_ * dt, 0.0], [s_ * dt, 0.0], [0.0, dt]])
        P = solve_discrete_are(A, Bm, Q, R)
        K = np.linalg.solve(R + Bm.T @ P @ Bm, Bm.T @ P @ A)
        e = x[b] - xr[b]
        e[2] = (e[2] + np.pi) % (2 * np.pi) - np.pi
        np.clip(ur[b] - K @ e, [-2.0, -3.0], [2.0, 3.0])
    return time.perf_counter() - t


def cfg2_scipy_baseline(B_total, seconds):
    """Config 2's SciPy leg: solve_discrete_are + np.linalg.solve over a
    bounded sample of the workload, a fork pool of the job's CPU share.  Runs before the GPU is
    initialised (worker processes are forked, never exec'ed)."""
    import multiprocessing as mp
    import numpy as np
    from oracle import figure8
    from rmpc import workloads as W
    threads = cpu_threads()
    n = max(threads * 8, int(seconds * threads * 1500))          # ~0.7 ms per robot per thread
    idx = np.linspace(0, B_total - 1, min(n, B_total)).astype(np.int64)
    xr, ur = figure8.offset_segments(2.0, 0.5, 0.02, W.t0_at(idx, B_total), 1)
    x = xr[:, 0] + W.noise_at(idx, W.CONFIGS["cfg2"]["seed"])
    parts = np.array_split(np.arange(len(idx)), threads)
    with mp.get_context("fork").Pool(threads) as pool:
        t = time.perf_counter()
        pool.map(_scipy_lqr_chunk, [(x[q], xr[q, 0], ur[q, 0]) for q in parts])
        wall = time.perf_counter() - t
    return {"value": len(idx) / wall, "unit": "controls/s", "cores": threads, "kind": "reference-arithmetic",
            "sample": f"{len(idx)} robots of the workload, SciPy {__import__('scipy').__version__} "
                      "solve_discrete_are + numpy.linalg.solve + control law per robot (lqr_controller.py:"
                      "116-132, 175-187), fork pool"}


def bench_other(args, world, rank, local, dist, pre=None):
    """BASELINE config 2 (batched LQR: DARE + gain + control per robot, no gain cache) and
    config 5 (one hybrid switching step: risk, dwell, LQR/MPC branches).  Same timing
    contract as config 3; one JSON line with the config's own unit of work."""
    import numpy as np
    import torch
    import rmpc
    from rmpc import workloads as W

    cfg = W.CONFIGS[args.config]
    B_per = cfg["B"]
    B_total = B_per * world
    idx = W.shard_indices(B_total, world, rank)        # round-robin, as config 3
    B = idx.size
    dev = torch.device(f"cuda:{local}")
    S = max(1, args.inflight)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream(device=dev) for _ in range(S - 1)]
    lp = rmpc._native.lqr_params([15, 15, 8], [.1, .1], 0.02, 2.0, 3.0, use_cache=False)
    if args.config == "cfg2":
        fleets = []                      # one fleet per slot in flight (rmpc.workloads.fleet_t0)
        for f in range(S):
            xr_f, ur_f = rmpc.batch.figure8_batch(W.fleet_t0(idx, B_total, f, S), 1, device=local)
            x_f = xr_f[:, 0] + W.noise_at(idx, W.fleet_seed(cfg["seed"], f))
            fleets.append((x_f, xr_f, ur_f))
        x_h, xr_h, ur_h = fleets[0]
        dfl = [(torch.from_numpy(a).to(dev), torch.from_numpy(np.ascontiguousarray(b[:, 0])).to(dev),
                torch.from_numpy(np.ascontiguousarray(c[:, 0])).to(dev)) for a, b, c in fleets]
        us = [torch.empty(B, 2, dtype=torch.float64, device=dev) for _ in range(S)]
        sts = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(S)]

        def step(k=0):
            i = k % S
            x, xr, ur = dfl[i]
            rmpc.batch.lqr_control_batch_dev(lp, x, xr, ur, us[i], status=sts[i], device=local,
                                             stream=streams[i], slot=i)
        metric, unit = "LQR control steps/sec (DARE + gain + control per robot, no cache)", "controls/s"
        flops_unit, bytes_unit = 6.0e3, 80.0
        workload = f"cfg2: compute_control_at_operating_point, Q=[15,15,8] R=[.1,.1], {B_per} robots/GPU"
    else:
        # ~half the robots within 0.767 m of an obstacle edge (MPC branch), half farther
        # (rmpc.workloads.cfg5_t0; tests/test_gpu_fullsize.py checks this exact workload)
        N = cfg["N"]
        # one fleet per slot in flight: fleet f's robots are the config's with other start
        # noise (the arc pools of cfg5_t0 fix which robots are near an obstacle)
        fleets = []
        for f in range(S):
            xr_f, ur_f = rmpc.batch.figure8_batch(W.cfg5_t0(idx), N + 1, device=local)
            x_f = xr_f[:, 0] + W.noise_at(idx, W.fleet_seed(cfg["seed"], f))
            fleets.append((torch.from_numpy(x_f).to(dev), torch.from_numpy(xr_f).to(dev),
                           torch.from_numpy(ur_f).to(dev), x_f))
        x_h, xr_h, ur_h = fleets[0][3], fleets[0][1].cpu().numpy(), fleets[0][2].cpu().numpy()
        obs = torch.tensor(W.DEFAULT_OBS, dtype=torch.float64, device=dev)
        mp = rmpc._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0,
                                     0.02, block_size=1)
        rp = rmpc._native.risk_params()
        # per in-flight slot: switch state, outputs (each slot is an independent fleet)
        states = [dict(prev_ctrl=torch.full((B,), -1, dtype=torch.int32, device=dev),
                       steps_since=torch.zeros(B, dtype=torch.int32, device=dev),
                       step_count=torch.full((B,), 10, dtype=torch.int32, device=dev),
                       cache=torch.zeros(B * rmpc._native.LQR_CACHE_DTYPE.itemsize, dtype=torch.uint8,
                                         device=dev)) for _ in range(S)]
        us = [torch.empty(B, 2, dtype=torch.float64, device=dev) for _ in range(S)]
        useds = [torch.empty(B, dtype=torch.uint8, device=dev) for _ in range(S)]
        risks = [torch.empty(B, dtype=torch.float64, device=dev) for _ in range(S)]
        used = useds[0]
        # The LQR branch without the gain cache (`lp` above, use_cache=False): in the reference
        # loop the reference index advances every step (run_simulation.py:525-526), so the
        # operating point moves and compute_gain's 1e-6 cache (lqr_controller.py:112-114) misses:
        # every LQR-branch robot solves its DARE every step.  Here the inputs repeat from step
        # to step, and a cache would turn every step after the first into a cached clip.

        # in flight, the MPC branch's first stage runs longer (scripts/r02_s3_caps_cfg.sh:
        # fast cap 9 against the single-batch default 6)
        # (config 5's side streams: on at three in flight, 398-418M against 233M steps/s without;
        # off at ten, whose 20 streams would oversubscribe the hardware queues -- profiles/r06)
        cset = W.inflight_settings("cfg5") if S > 1 else dict(W.ALONE)
        if args.stage_caps:
            cset["caps"] = tuple(int(v) for v in args.stage_caps.split(","))
        if args.stage_passes:
            cset["passes"] = tuple(int(v) for v in (args.stage_passes + ",0").split(",")[:2])
        if S > 1:
            cset["cold_start"] = args.cold_start
            if args.inflight_side is not None:
                cset["side"] = bool(args.inflight_side)
        caps = cset["caps"]
        for i in range(S):
            rmpc.batch.configure(cset, device=local, slot=i)

        def step(k=0):
            i = k % S
            x, xr, ur, _ = fleets[i]
            rmpc.batch.hybrid_step_batch_dev(rp, lp, mp, x, xr, ur, obs, states[i], us[i], useds[i], risks[i],
                                             device=local, stream=streams[i], slot=i)
        metric, unit = "hybrid LQR/MPC control steps/sec (risk + dwell switch + branch)", "steps/s"
        flops_unit, bytes_unit = None, None
        workload = (f"cfg5: run_hybrid_simulation step, N={N}, 3 obstacles, ~50% of robots within "
                    f"0.767 m of an obstacle edge, {B_per} robots/GPU")
    elapsed, (k_ms, k_evt_ms) = _timed(args, step, dist, dev, S)
    k_avg_s = k_ms / 1e3
    alone_default_s = None
    if args.config == "cfg5" and caps[0]:
        # one batch alone with the library's default caps (what one batch at a time would use)
        torch.cuda.synchronize()
        rmpc.batch.configure(dict(W.ALONE, side=bool(args.alone_side)), device=local, slot=0)
        alone_default_s = alone_times(lambda: step(0), torch.cuda.current_stream(), args.steps)[0] / 1e3
        rmpc.batch.configure(cset, device=local, slot=0)
    k_roof_s = alone_default_s or k_avg_s     # the roofline's launch: one batch alone, library defaults
    elapsed, _ = W.aggregate(dist, elapsed, [], device=coll_device(args, dev))
    line = {"metric": metric, "value": B_total * args.steps / elapsed,
            "value_one_batch_alone": B_total / (alone_default_s or k_avg_s), "unit": unit, "n_gpus": world,
            **({"value_one_batch_alone_inflight_caps": B_total / k_avg_s} if alone_default_s else {}),
            "schema": SCHEMA,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: Figure-8 references at per-robot time offsets + seeded start noise",
            "config": {"workload": workload, "robots_per_gpu": B_per, "global_batch": B_total,
                       "parallelism": parallelism(args, world), "batches_in_flight": S}}
    if args.config == "cfg5":
        line["config"]["stage_caps"] = list(caps) if caps[0] else "library default"
        line["config"]["alone_side_stream"] = bool(args.alone_side)
    if flops_unit:
        ach = flops_unit * B / k_roof_s / 1e12
        line["roofline"] = {"bound": "valu-fp64", "achieved": ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                            "frac": ach / FP64_PEAK_TFLOPS, "traffic": None,
                            "kernel": "lqr_control_kernel", "kernel_avg_ms": k_roof_s * 1e3,
                            "flops_per_unit": flops_unit, "algorithmic_bytes_per_unit": bytes_unit,
                            "hbm_gbs_algorithmic": bytes_unit * B / k_roof_s / 1e9,
                            "note": "launch-latency bound at this batch (one ~10-15 us kernel)"}
    else:
        used_h = used.cpu().numpy().astype(bool)
        fm = float(used_h.mean())
        line["mpc_fraction"] = fm
        line["kernel_avg_ms"] = k_roof_s * 1e3
        # closed loop (rank 0, N=1; never `value`): run_simulation.py's hybrid loop on the device,
        # cold and with the warm start across calls (the MPC branch's robots, per-robot stamps)
        if world == 1 and rank == 0 and not args.no_closed_loop:
            line["closed_loop"] = closed_loop(dev, B, W.DEFAULT_OBS, N, False, hybrid=True, t0=W.cfg5_t0(idx))
            line["closed_loop"]["unit"] = "hybrid control steps/s"

        # risk 10 n_o + the chosen branch's canonical work per robot
        # (MPC: condensed-QP model at the MPC robots' mean iterations; LQR: 6e3)
        its_mpc = None
        try:
            sc = np.full(int(used_h.sum()), 10, np.int32)
            sel = np.where(used_h)[0]
            o = rmpc.batch.mpc_solve_batch(mp, x_h[sel], xr_h[sel], ur_h[sel], W.DEFAULT_OBS, step_count=sc,
                                           device=local, want_seq=False)
            its_mpc = float(o["iters"].mean())
        except Exception:   # noqa: BLE001  (diagnostic only)
            its_mpc = 2.2
        f_unit = 10 * 3 + fm * canonical_flops(N, 3, its_mpc) + (1 - fm) * 6.0e3
        ach = f_unit * B / k_roof_s / 1e12
        line["roofline"] = {"bound": "valu-fp64", "achieved": ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                            "frac": ach / FP64_PEAK_TFLOPS, "traffic": None,
                            "kernel": "hybrid_decide_kernel + lqr_control_kernel + MPC pipeline (compacted lists)",
                            "kernel_avg_ms": k_roof_s * 1e3, "flops_per_unit_canonical": f_unit,
                            "mpc_iters_mean": its_mpc,
                            "hbm_gbs_algorithmic": (24 + fm * algorithmic_bytes(N, 3, False) + (1 - fm) * 80) * B
                            / k_roof_s / 1e9}
        pmc_into_roofline(line["roofline"], "_cfg5", (24 + fm * algorithmic_bytes(N, 3, False) + (1 - fm) * 80) * B,
                          k_roof_s)
    # ---- CPU baseline (rank 0, N=1): the oracle's C restatement of the same step
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        from oracle import cpu
        threads = cpu_threads()
        lq = cpu.lqr_params((15, 15, 8), (.1, .1), 0.02, 2.0, 3.0, use_cache=0)
        if args.config == "cfg2":
            xr0, ur0 = np.ascontiguousarray(xr_h[:, 0]), np.ascontiguousarray(ur_h[:, 0])
            cpu.lqr_control_batch(lq, x_h, xr0, ur0, threads=threads)
            reps, t_c = 0, 0.0
            while t_c < args.cpu_seconds * 0.5 and reps < 4000:
                t = time.perf_counter()
                cpu.lqr_control_batch(lq, x_h, xr0, ur0, threads=threads)
                t_c += time.perf_counter() - t
                reps += 1
            line["cpu_baseline"] = {"value": B * reps / t_c, "unit": "controls/s", "cores": threads, "kind": "port",
                                    "sample": f"the whole {B}-robot batch x {reps} reps (oracle/c SDA DARE + gain + "
                                              "control, OpenMP)", "host": host_info()}
            if pre is not None:
                line["cpu_baseline_scipy"] = pre
        else:
            # risk + dwell (the first step: the risk decides) + branches, on a strided sample
            nsamp = min(B, 16384)
            sl = slice(0, B, B // nsamp)
            xs, xrs, urs = x_h[sl], xr_h[sl], ur_h[sl]
            cp = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
            lq = cpu.lqr_params((15, 15, 8), (.1, .1), 0.02, 2.0, 3.0, use_cache=0)   # as the GPU leg

            def cpu_step():
                d = np.min([np.hypot(xs[:, 0] - ox, xs[:, 1] - oy) - r for ox, oy, r in W.DEFAULT_OBS], 0)
                rk = np.clip(1.0 - (d - 0.3) / (1.0 - 0.3), 0.0, 1.0)          # risk_metrics.py:84-129
                m = 0.6 * rk >= 0.2                                           # :212 (alpha normalised)
                im, il = np.where(m)[0], np.where(~m)[0]
                cpu.mpc_solve_batch(cp, xs[im], xrs[im], urs[im], W.DEFAULT_OBS,
                                    step_count=np.full(len(im), 10, np.int32), threads=threads)
                cpu.lqr_control_batch(lq, xs[il], np.ascontiguousarray(xrs[il, 0]),
                                      np.ascontiguousarray(urs[il, 0]), threads=threads)
            cpu.set_pdas_caps(6, 4)        # the switch's MPC branch: fast cap 6, 4 tail solves
            cpu_step()
            reps, t_c = 0, 0.0
            while t_c < args.cpu_seconds * 0.8 and reps < 1000:
                t = time.perf_counter()
                cpu_step()
                t_c += time.perf_counter() - t
                reps += 1
            cpu.set_pdas_caps(0, 0)
            line["cpu_baseline"] = {"value": nsamp * reps / t_c, "unit": "steps/s", "cores": threads, "kind": "port",
                                    "sample": f"{nsamp} robots (every {B // nsamp}th) x {reps} reps: numpy risk + "
                                              "dwell, oracle/c MPC on the MPC branch and SDA LQR on the rest (OpenMP)",
                                    "host": host_info()}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
