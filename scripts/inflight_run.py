"""Minimal in-flight run of the MPC pipeline for counter passes (diagnostics): S fleets of a
BASELINE configuration in flight on their own contexts and streams, exactly as bench.py's timed
loop sets them up (rmpc.workloads.INFLIGHT: stage caps, zero-correction first sets, stage
passes, lanes per robot, side streams), and nothing else -- no one-batch-alone legs, no host-pointer or closed-loop calls -- so that every
dispatch of the MPC kernels in a rocprofv3 pass belongs to the in-flight pipeline.
Usage: python scripts/inflight_run.py [--config cfg3|cfg4]
       [--inflight S] [--steps 16] [--warmup 8] [--caps F,T] [--passes c1[,c2]]
Prints one JSON line: wall-clock rate of the timed steps and the solver status counts."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3", choices=["cfg3", "cfg4"])
    ap.add_argument("--inflight", type=int, default=None, help="default: bench.py's (config 3: 10, config 4: 8)")
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--caps", default=None)
    ap.add_argument("--passes", default=None, help="rmpc_ctx_set_stage_passes on the in-flight contexts")
    ap.add_argument("--hw-queues", type=int, default=None, help="default: bench.py's (config 3: 32, config 4: 16)")
    args = ap.parse_args()
    if args.inflight is None:
        args.inflight = 10 if args.config == "cfg3" else 8
    if args.hw_queues is None:
        args.hw_queues = 32 if args.config == "cfg3" else 16
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    import numpy as np
    import torch
    import rmpc
    from rmpc import workloads as W
    dev = torch.device("cuda:0")
    cfg = W.CONFIGS[args.config]
    N, obs_list, seed = cfg["N"], cfg["obs"], cfg["seed"]
    B = cfg["B"] if args.config == "cfg3" else 32768
    f32 = args.config == "cfg4"
    idx = np.arange(B)
    S = args.inflight
    fleets, outs, counts = [], [], []
    for f in range(S):
        xr, ur = rmpc.batch.figure8_batch(W.fleet_t0(idx, B, f, S), N + 1, device=0)
        x0 = xr[:, 0] + W.noise_at(idx, W.fleet_seed(seed, f))
        fleets.append([torch.from_numpy(a).to(dev) for a in (x0, xr, ur)])
        outs.append(dict(u0=torch.empty(B, 2, dtype=torch.float64, device=dev),
                         u_seq=torch.empty(B, N, 2, dtype=torch.float64, device=dev),
                         x_pred=torch.empty(B, N + 1, 3, dtype=torch.float64, device=dev),
                         cost=torch.empty(B, dtype=torch.float64, device=dev),
                         status=torch.empty(B, dtype=torch.int32, device=dev),
                         slack_used=torch.empty(B, dtype=torch.uint8, device=dev),
                         iters=torch.empty(B, dtype=torch.int32, device=dev)))
        counts.append(torch.full((B,), 10, dtype=torch.int32, device=dev))
    obs = torch.tensor(obs_list, dtype=torch.float64, device=dev).reshape(-1, 3)
    p = rmpc._native.mpc_params(N, [15, 15, 50], [.1, .1], [30, 30, 40], 0.3, 5000.0, 2.0, 3.0, 0.02,
                                precision=1 if f32 else 0)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream(device=dev) for _ in range(S - 1)]
    cset = W.inflight_settings(args.config) if S > 1 else dict(W.ALONE)     # bench.py's settings
    if args.caps:
        cset["caps"] = tuple(int(v) for v in args.caps.split(","))
    if args.passes:
        cset["passes"] = tuple(int(v) for v in (args.passes + ",0").split(",")[:2])
    for i in range(S):
        rmpc.batch.configure(cset, device=0, slot=i)

    def step(k):
        i = k % S
        x0, xr, ur = fleets[i]
        rmpc.batch.mpc_solve_batch_dev(p, x0, xr, ur, obs, outs[i], step_count=counts[i], device=0,
                                       stream=streams[i], slot=i)

    for k in range(max(args.warmup, S)):
        step(k)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    st = torch.cat([o["status"] for o in outs]).cpu().numpy()
    its = torch.cat([o["iters"] for o in outs]).cpu().numpy()
    print(json.dumps({"config": args.config, "inflight": S, "steps": args.steps, "settings": cset,
                      "value": B * args.steps / el,
                      "ms_per_step": el / args.steps * 1e3, "optimal": int((st == 0).sum()), "robots": int(st.size),
                      "iters_mean": float(its.mean())}), flush=True)


if __name__ == "__main__":
    main()
