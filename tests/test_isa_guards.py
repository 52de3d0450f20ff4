"""ISA guards of the product kernels that write M0 themselves (CPU: hipcc cross-compiles gfx950).

lsqp4_kernel.hip issues its LDS-DMAs (`global_load_lds_dword[x4]`) from inline asm that loads
the LDS destination into M0.  Two rules keep that correct without saving M0 around every DMA
(saving it cost c5 1.5-2.5 %, profiles/r03_dma_asm_ab.txt):
  * the SALU write of M0 and the DMA reading it are one wait state apart (`s_nop 0`); a
    second DMA of the same asm block (the other half of a strip) reuses that M0;
  * the compiler itself never touches M0 in these kernels, so nothing it emits can see the
    value the asm leaves there (checked here on the generated code, so a compiler or source
    change that starts using M0 fails this test instead of corrupting LDS silently).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mpistragglers.jl_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _asm(tmp_path, src):
    out = tmp_path / (os.path.basename(src) + ".s")
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--offload-device-only", "-S",
           "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, os.path.join(CSRC, src), "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    return out.read_text()


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_lsqp4_m0_writes_are_separated_and_private(tmp_path):
    text = _asm(tmp_path, "lsqp4_kernel.hip")
    in_asm = m0_in_block = False
    prev = None
    m0_writes = dma = 0
    for raw in text.splitlines():
        line = raw.split(";")[0].strip()
        if raw.strip().startswith(";;#ASMSTART"):
            in_asm, prev, m0_in_block = True, None, False
            continue
        if raw.strip().startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not line or line.startswith("."):
            continue
        mentions_m0 = re.search(r"\bm0\b", line) is not None
        if not in_asm:
            assert not mentions_m0, f"compiler-emitted instruction uses M0: {line}"
            continue
        if line.startswith("s_mov_b32 m0,"):
            m0_writes += 1
        if line.startswith("global_load_lds"):
            dma += 1
            # the first DMA after an M0 write sits one wait state behind it; further DMAs of
            # the same asm block (a strip's two halves) reuse that M0 value
            assert prev == "s_nop 0" or (prev or "").startswith("global_load_lds"), \
                f"LDS-DMA right after the M0 write without a wait state: {prev!r} -> {line}"
            assert m0_in_block, f"LDS-DMA in an asm block that did not set M0: {line}"
        if line.startswith("s_mov_b32 m0,"):
            m0_in_block = True
        prev = line
    assert m0_writes > 0 and m0_writes <= dma <= 2 * m0_writes


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_lsq_kernels_use_no_scratch(tmp_path):
    """Every lsq_grad_kernel variant (the fused head and pre-armed ones included) runs without
    scratch: a pointer that could point at either the kernel-argument EpochArgs or its LDS copy
    once made the compiler copy the 976-B struct to scratch, 3.5 KiB per workgroup and 50 us per
    c1 launch (profiles/r03_c1_head_ab.txt)."""
    text = _asm(tmp_path, "lsq_kernel.hip")
    sizes = re.findall(r"\.private_segment_fixed_size:\s*(\d+)", text)
    names = re.findall(r"\.name:\s*(_Z\S*lsq_grad_kernel\S*)", text)
    assert names and len(sizes) >= len(names), (len(names), len(sizes))
    assert all(int(s) == 0 for s in sizes), sizes
