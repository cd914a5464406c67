"""bench.py's JSON contract on the GPU (the driver parses this line at every round's end).

Short runs of the headline configuration and of configs 4 and 5 (a few steps, the CPU
baseline on a one-second budget, no closed loops / drop-in / host-pointer legs): exactly one
JSON line with the contract's fields, the roofline and cpu_baseline objects, every robot
optimal, and the settings the line reports equal to rmpc.workloads.INFLIGHT's.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config")


def _bench(args):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "RMPC_DIAG", "RMPC_LIB_PATH"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("config", ["cfg3", "cfg4", "cfg5"])
def test_bench_line_contract(gpu_lib, config):
    from rmpc import workloads as W
    d = _bench(["--config", config, "--steps", "4", "--warmup", "2", "--cpu-seconds", "1", "--no-pcie",
                "--no-closed-loop", "--no-drop-in"])
    for k in CONTRACT:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["value"] > 0 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["data"].startswith("synthetic")
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port" and cb["sample"]
    st = W.inflight_settings(config)
    assert d["config"]["batches_in_flight"] == (10 if config in ("cfg3", "cfg5") else 8)
    assert d["config"]["stage_caps"] == list(st["caps"])
    if config == "cfg5":
        assert d["unit"] == "steps/s"
        return
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"])
    assert d["config"]["stage_passes"] == (list(st["passes"]) if st["passes"][0] else "one pass")
    assert d["solver"]["optimal"] == d["config"]["robots_per_gpu"]
    assert d["max_abs_du_vs_cpu_port"] <= 1e-9
    if config == "cfg3":
        assert r["frac_executed_in_flight"] > 0 and r["traffic"] > 0
