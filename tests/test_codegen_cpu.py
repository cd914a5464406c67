"""Code-generation guard for the lane-per-robot MPC kernel (no GPU needed).

The ROCm 7.2 compiler (AMD clang 22.0.0git roc-7.2.0) has dropped the whole output pass of
`fast_body` (rmpc_fast_body.h) from `mpc_ltv_fast_kernel` for some source forms of the
hand-on condition that are logically identical to the shipped one: the LLVM IR still holds the
output stores, and the backend's branch folding removes them (HISTORY.md section 10).  Such a
build still returns correct answers -- every robot then reaches the tail as if uncertified --
at a third of the speed, so no parity test notices.  This test reads the device code of the
built library and checks that every instance of the kernel still stores 64- or 128-bit
values (u0, u_seq, x_pred): the hand-on path alone stores only 32-bit words.
"""
import os
import re
import subprocess

import pytest

from conftest import PKG_DIR

LLVM_BIN = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def library_path():
    return os.environ.get("RMPC_LIB_PATH") or os.path.join(PKG_DIR, "rmpc", "librmpc.so")


def device_functions(so, tmp):
    """{function name: [instruction mnemonics]} over every gfx950 code object in `so`."""
    tools = [os.path.join(LLVM_BIN, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]
    if not all(os.path.exists(t) for t in tools):
        pytest.skip("ROCm LLVM tools not found")
    objcopy, bundler, objdump = tools
    fat = tmp / "fatbin.bin"
    subprocess.run([objcopy, f"--dump-section=.hip_fatbin={fat}", so, str(tmp / "copy.so")], check=True)
    blob = fat.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
    if not starts:      # a compressed bundle (CCOB) or another layout: nothing to read here
        pytest.skip("no uncompressed offload bundle in .hip_fatbin")
    if TARGET.encode() not in blob:
        pytest.skip(f"library built without {TARGET} (Makefile ARCH override)")
    funcs = {}
    for i, s in enumerate(starts):
        part = tmp / f"bundle{i}.bin"
        part.write_bytes(blob[s:starts[i + 1] if i + 1 < len(starts) else len(blob)])
        if TARGET.encode() not in part.read_bytes():
            continue
        co = tmp / f"bundle{i}.co"
        subprocess.run([bundler, "--unbundle", "--type=o", f"--input={part}", f"--targets={TARGET}",
                        f"--output={co}"], check=True)
        dis = subprocess.run([objdump, "-d", "--no-show-raw-insn", str(co)], check=True,
                             capture_output=True, text=True).stdout
        name = None
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                name = m.group(1)
                funcs[name] = []
            elif name and line.startswith("\t"):
                funcs[name].append(line.split()[0])
    return funcs


def test_fast_kernel_instances_keep_their_output_pass(tmp_path):
    so = library_path()
    if not os.path.exists(so):
        pytest.skip("librmpc.so not built")
    funcs = device_functions(so, tmp_path)
    fast = {n: ops for n, ops in funcs.items() if "mpc_ltv_fast_kernel" in n}
    assert len(fast) >= 10, sorted(funcs)
    missing = [n for n, ops in fast.items()
               if not any(op in ("global_store_dwordx2", "global_store_dwordx4") for op in ops)]
    assert not missing, f"output stores missing from {missing}"
