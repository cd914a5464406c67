"""C-ABI surface checks that need no GPU: symbols, struct layout, error paths, params.yaml."""
import ctypes as C
import os
import re
import subprocess
import textwrap

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

HEADER = os.path.join(ROOT, "include", "rmpc.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rmpc_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(lib):
    names = header_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    from rmpc import _native
    assert set(names) == set(_native.exported_symbols())


def test_abi_version(lib):
    assert lib.rmpc_abi_version() == 1


def test_struct_layout_matches_header(tmp_path):
    """Compile a probe against include/rmpc.h and compare sizeof/offsetof with ctypes."""
    from rmpc import _native as n
    probe = tmp_path / "probe.c"
    probe.write_text(textwrap.dedent(f"""
        #include <stdio.h>
        #include <stddef.h>
        #include "{HEADER}"
        int main(void) {{
          printf("%zu %zu %zu %zu\\n", sizeof(RmpcMpcParams), sizeof(RmpcLqrParams),
                 sizeof(RmpcRiskParams), sizeof(RmpcLqrCache));
          printf("%zu %zu %zu %zu\\n", offsetof(RmpcMpcParams, Q), offsetof(RmpcMpcParams, dt),
                 offsetof(RmpcLqrParams, max_iter), offsetof(RmpcLqrCache, valid));
          printf("%zu %zu %zu\\n", sizeof(RmpcRolloutParams), offsetof(RmpcRolloutParams, dt),
                 offsetof(RmpcRolloutParams, omega_max));
          return 0; }}"""))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", str(probe), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    got = [int(v) for v in out]
    want = [C.sizeof(n.MpcParams), C.sizeof(n.LqrParams), C.sizeof(n.RiskParams),
            C.sizeof(n.LqrCache), n.MpcParams.Q.offset, n.MpcParams.dt.offset,
            n.LqrParams.max_iter.offset, n.LqrCache.valid.offset,
            C.sizeof(n.RolloutParams), n.RolloutParams.dt.offset, n.RolloutParams.omega_max.offset]
    assert got == want
    assert n.LQR_CACHE_DTYPE.itemsize == C.sizeof(n.LqrCache)


def test_null_context_is_rejected(lib):
    from rmpc import _native as n
    p = n.mpc_params(20, [15, 15, 50], [.1, .1], [30, 30, 40], .3, 5000., 2., 3., .02)
    rc = lib.rmpc_mpc_solve_batch(None, C.byref(p), 1, None, None, 21, None, 21, None, 0, None,
                                  None, None, None, None, None, None, None)
    assert rc == -1
    assert b"ctx" in lib.rmpc_last_error()
    lp = n.lqr_params([15, 15, 8], [.1, .1], .02, 2., 3.)
    assert lib.rmpc_lqr_control_batch(None, C.byref(lp), 1, None, None, None, None, None, None,
                                      None, None, None) == -1
    assert lib.rmpc_ctx_destroy(None) == 0
    assert lib.rmpc_ctx_set_stage_caps(None, 9, 4) == -1
    assert lib.rmpc_ctx_set_side_stream(None, 1) == -1
    assert lib.rmpc_ctx_set_cold_start(None, 1) == -1
    assert lib.rmpc_ctx_set_stage_passes(None, 1, 0) == -1
    assert lib.rmpc_ctx_set_lanes_per_robot(None, 1) == -1
    assert lib.rmpc_ctx_set_warm_start(None, 1) == -1


def test_context_without_device_fails_loudly(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from rmpc import _native as n
    with pytest.raises(n.RmpcError):
        n.context(0)


LLVM_BIN = "/opt/rocm/lib/llvm/bin"


def gfx950_code_objects(so_path, tmp_path):
    """The gfx950 code objects embedded in a HIP shared library: its .hip_fatbin section holds
    one clang offload bundle per translation unit (magic, entry count, then per entry offset,
    size, target-triple length and triple)."""
    import struct
    sec = tmp_path / "fatbin.bin"
    subprocess.run([f"{LLVM_BIN}/llvm-objcopy", "--dump-section", f".hip_fatbin={sec}", so_path,
                    str(tmp_path / "stripped.so")], check=True)
    b = sec.read_bytes()
    magic, pos, out = b"__CLANG_OFFLOAD_BUNDLE__", 0, []
    while (i := b.find(magic, pos)) >= 0:
        n, q = struct.unpack_from("<Q", b, i + 24)[0], i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", b, q)
            triple = b[q + 24: q + 24 + tl].decode()
            q += 24 + tl
            if triple.endswith("gfx950"):
                out.append(b[i + off: i + off + size])
        pos = i + 1
    return out


def test_library_has_no_packed_fp32_code(lib, tmp_path):
    """The shipped library holds no packed-fp32 (VOP3P v_pk_{fma,mul,add}_f32) instructions.
    In round 2 an fp32 build with packed code certified wrong controls for 29-32 of 2048 robots
    (lanes 12-15 of lane rows 1-3) depending on the instruction schedule; the library is built
    with -fno-slp-vectorize -fno-vectorize, the two passes that emitted packed fp32 (the
    Makefile; HISTORY.md section 4).  This guards against a toolchain update or a code change
    bringing such code back unnoticed."""
    if not os.path.exists(f"{LLVM_BIN}/llvm-objdump"):
        pytest.skip("no llvm-objdump")
    from rmpc import _native
    cos = gfx950_code_objects(_native.LIB_PATH, tmp_path)
    assert len(cos) >= 4                          # one per device translation unit
    found = {}
    for k, co in enumerate(cos):
        f = tmp_path / f"co{k}.elf"
        f.write_bytes(co)
        dis = subprocess.run([f"{LLVM_BIN}/llvm-objdump", "-d", "--mcpu=gfx950", str(f)], check=True,
                             capture_output=True, text=True).stdout
        assert "mpc_" in dis or "lqr_" in dis or "kernel" in dis
        for m in re.findall(r"\bv_pk_(?:fma|mul|add)_f32\b", dis):
            found[m] = found.get(m, 0) + 1
    assert not found, found


def test_params_yaml_surface():
    from rmpc import params
    cfg = params.load_params(os.path.join(GOLDEN, "params.yaml"))
    lk = params.lqr_kwargs(cfg)
    mk = params.mpc_kwargs(cfg)
    assert lk == dict(Q_diag=[10.0, 10.0, 1.0], R_diag=[0.1, 0.1], dt=0.02, v_max=1.0,
                      omega_max=1.5)
    assert mk["horizon"] == 10 and mk["slack_penalty"] == 1000.0 and mk["solver"] == "ECOS"
    assert mk["P_diag"] == [20.0, 20.0, 2.0]
    s = params.mpc_struct(cfg)
    assert s.horizon == 10 and list(s.Q) == [10.0, 10.0, 1.0]
