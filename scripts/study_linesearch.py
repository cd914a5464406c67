"""Round-4 model study: would a line search with several trial points up front shorten the hardest
robots' projected-Newton phase?  CPU only, oracle code (test infrastructure).

The C port staged like the device (config 3: caps (7, 4); config 4: (12, 6)) follows the GPU
pipeline's iterate path robot by robot.  Study builds of it (RMPC_LS_STUDY, oracle/c/rmpc_cpu.c)
replace the Armijo backtracking by four (or 200) trial step lengths along the projection arc,
taking the lowest objective among those that pass the Armijo test (falling back to the
backtracking when none does).  Reported: the iteration histogram's tail (the robots that set the
tail launch's length), the projected-Newton iterations and objective evaluations in all, and
the largest control difference against the default build (the certified optimum is the same).
Usage: python scripts/study_linesearch.py   (builds /tmp/ls_<mode>.so with gcc first)"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "risk-aware-hybrid-lqr-mpc-navigation-for-autonomous-systems_amd")]
from oracle import cpu, figure8  # noqa: E402
from rmpc import workloads as W  # noqa: E402

MODES = {0: "Armijo + quadratic interpolation (default)", 1: "best of {1, 1/2, 1/4, 1/8}",
         2: "best of {2, 1, 1/2, 1/4}", 3: "best of {1.5, 1, 0.7, 0.45}", 4: "best of 200 on (0, 2] (ceiling)"}


def build(mode):
    path = f"/tmp/ls_{mode}.so"
    src = os.path.join(ROOT, "oracle", "c", "rmpc_cpu.c")
    subprocess.run(["gcc", "-O3", "-march=x86-64-v3", "-fopenmp", "-fPIC", "-std=c11", f"-DRMPC_LS_STUDY={mode}",
                    "-shared", "-o", path, src, "-lm"], check=True)
    return path


def run(cfg_name, B, caps):
    cfg = W.CONFIGS[cfg_name]
    N, obs = cfg["N"], cfg["obs"]
    idx = np.arange(B)
    xr, ur = figure8.offset_segments(2.0, 0.5, 0.02, W.t0_at(idx, B), N + 1)
    x0 = xr[:, 0] + W.noise_at(idx, cfg["seed"])
    cp = cpu.mpc_params(N, (15, 15, 50), (.1, .1), (30, 30, 40), 0.3, 5000., 2., 3., 0.02)
    lib = cpu.lib()
    lib.rmpc_cpu_reset_counters()
    cpu.set_pdas_caps(*caps)
    r = cpu.mpc_solve_batch(cp, x0, xr, ur, obs, step_count=np.full(B, 10, np.int32), threads=8)
    cpu.set_pdas_caps(0, 0)
    lib.rmpc_cpu_counter.restype = C.c_long
    return r, [lib.rmpc_cpu_counter(i) for i in range(3)]


def main():
    cases = [("cfg3", 65536, (7, 4)), ("cfg4", 32768, (12, 6))]
    base = {}
    for mode in MODES:
        cpu._LIB = None if mode == 0 else C.CDLL(build(mode))
        if mode == 0:
            cpu.lib()
        for name, B, caps in cases:
            r, cnt = run(name, B, caps)
            its = r["iters"]
            if mode == 0:
                base[name] = r
                du = 0.0
            else:
                du = float(np.abs(r["u_seq"] - base[name]["u_seq"]).max())
            q = np.sort(its)[::-1]
            print(f"{name} mode {mode} ({MODES[mode]}): status {np.bincount(r['status'], minlength=3).tolist()} "
                  f"max {its.max()} top-10 {q[:10].tolist()} p99.9 {np.percentile(its, 99.9):.0f} | "
                  f"PN iterations {cnt[1]} F evaluations {cnt[2]} | max |du| vs default {du:.1e}", flush=True)
    cpu._LIB = None


if __name__ == "__main__":
    main()
