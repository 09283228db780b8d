"""The shipped gfx950 code has no packed-FP32 VALU ops (CPU only: disassembles libkrrn_hip.so).

DESIGN.md section 5: a packed-FP32 result (v_pk_mul_f32 / v_pk_fma_f32) in the surface gather-conv
came out wrong while the split-bf16 Winograd ran on the same CU, and the library is built with
`-Xclang -target-feature -Xclang -packed-fp32-ops` (csrc/Makefile) so that none is emitted. This
test guards that flag: a compiler upgrade, a new .hip file with its own flags or inline assembly
that brought the instructions back would fail here, before any GPU run."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "pose_estimation_amd", "libkrrn_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"
PACKED_F32 = re.compile(r"\bv_pk_(fma|mul|add|mov)_[bf]32\b")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _code_objects(tmp):
    """The gfx950 code object of every source's offload bundle in the library's .hip_fatbin."""
    fat = os.path.join(tmp, "fat.bin")
    subprocess.check_call([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", LIB, os.devnull])
    data = open(fat, "rb").read()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    cos = []
    for i, o in enumerate(offs):
        b = os.path.join(tmp, f"b{i}.bin")
        open(b, "wb").write(data[o:offs[i + 1] if i + 1 < len(offs) else len(data)])
        co = os.path.join(tmp, f"b{i}.co")
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={b}",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        cos.append(co)
    return cos


@pytest.mark.skipif(not (os.path.exists(LIB) and shutil.which(f"{LLVM}/llvm-objdump")),
                    reason="library not built / no llvm-objdump")
def test_no_packed_fp32_valu_in_library(tmp_path):
    cos = _code_objects(str(tmp_path))
    csrc = os.path.join(ROOT, "pose_estimation_amd", "csrc")
    srcs = [f for f in os.listdir(csrc) if f.endswith(".hip") and "__global__" in open(os.path.join(csrc, f)).read()]
    assert len(cos) >= len(srcs), (len(cos), len(srcs))  # one bundle per source file with kernels
    kernels = 0
    for co in cos:
        asm = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                             capture_output=True, text=True).stdout
        kernels += len(re.findall(r"^[0-9a-f]+ <\S+>:$", asm, re.M))
        hits = [ln.strip() for ln in asm.splitlines() if PACKED_F32.search(ln)]
        assert not hits, (os.path.basename(co), hits[:5])
    assert kernels > 50, kernels
