"""Executed flops and VALU occupancy per library call from rocprofv3 --pmc passes.

Usage: python scripts/pmc_flops.py gpurun_out/<tag> out.json [entry-kernel substring]

fp64 flops = 64 x (2 FMA + ADD + MUL + TRANS) per wave instruction (SQ_INSTS_VALU_*_F64 count
wave-level instructions; exec-masked lanes are counted, so this is an upper bound); fp32 the same
with the *_F32 counters (config 4's fp32 pass).  SQ cycle counters are per-SE sums; only their
ratios are used: VALU active = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, waiting = SQ_WAIT_ANY /
SQ_WAVE_CYCLES.  Per launch = summed over every dispatch of the call's kernels, divided by the
dispatches of its entry kernel (scripts/pmc_common.py).
"""
import json
import sys

from pmc_common import per_launch

tag, out = sys.argv[1], sys.argv[2]
entry = sys.argv[3] if len(sys.argv) > 3 else "mpc_ltv_fast_kernel"
ks, launches, per = per_launch(tag, entry)


def fl(d, p):
    return 64 * (2 * d.get(f"SQ_INSTS_VALU_FMA_{p}", 0.0) + d.get(f"SQ_INSTS_VALU_ADD_{p}", 0.0)
                 + d.get(f"SQ_INSTS_VALU_MUL_{p}", 0.0) + d.get(f"SQ_INSTS_VALU_TRANS_{p}", 0.0))


res = {"note": __doc__.split("\n\n")[1].replace("\n", " "), "entry": entry, "kernels": {}}
t64 = t32 = 0.0
for k, d in ks.items():
    wc = d.get("SQ_WAVE_CYCLES", 0.0)
    res["kernels"][k] = {"fp64_flops": fl(d, "F64"), "fp32_flops": fl(d, "F32"), "valu_insts": d.get("SQ_INSTS_VALU"),
                         "waves": d.get("SQ_WAVES"), "dispatches_per_launch": per[k],
                         "valu_active_frac": d.get("SQ_ACTIVE_INST_VALU", 0.0) / wc if wc else None,
                         "wait_any_frac": d.get("SQ_WAIT_ANY", 0.0) / wc if wc else None,
                         "wait_inst_frac": d.get("SQ_WAIT_INST_ANY", 0.0) / wc if wc else None}
    t64 += fl(d, "F64")
    t32 += fl(d, "F32")
res["fp64_flops_per_launch"] = t64
res["fp32_flops_per_launch"] = t32
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
