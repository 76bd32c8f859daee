"""CPU check of the shipped code object (no GPU): the recurrence kernels that must own their
SIMD do.  The PLL chain and the biquad bank claim the whole register file (512 VGPRs incl.
AGPRs per wave, occupancy 1), so no wave of another kernel -- an MFMA FIR bank running on
another stream -- can share their SIMD; round 5 measured wrong PLL results (lanes 48-63 of a
packed-f32 mixer) when two MFMA bank waves shared the chain wave's SIMD (DESIGN.md 3.6,
profiles/r05_chain_probe.txt).  Reads the amdhsa kernel metadata of libsdrgpu.so's gfx950 code
objects with the ROCm LLVM tools."""
import os
import re
import struct
import subprocess

import pytest

from conftest import ROOT

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(ROOT, "unnamed-rust-sdr_amd", "libsdrgpu.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def kernel_registers(tmp_path):
    """{kernel symbol: (.vgpr_count, .agpr_count)} over every gfx950 code object bundled in the
    library's .hip_fatbin section (one clang offload bundle per translation unit)."""
    sec = tmp_path / "fatbin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={sec}", LIB,
                    str(tmp_path / "copy.so")], check=True)
    data = sec.read_bytes()
    regs, pos = {}, 0
    while (i := data.find(MAGIC, pos)) >= 0:
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" not in triple or not size:
                continue
            co = tmp_path / "co"
            co.write_bytes(data[i + off:i + off + size])
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)],
                                   capture_output=True, text=True, check=True).stdout
            for blk in notes.split("  - .agpr_count")[1:]:
                name = re.search(r"\.name:\s+(\S+)", blk).group(1)
                agpr = int(re.match(r":\s+(\d+)", blk).group(1))
                vgpr = int(re.search(r"\.vgpr_count:\s+(\d+)", blk).group(1))
                regs[name] = (vgpr, agpr)
        pos = i + len(MAGIC)
    return regs


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(f"{LLVM}/llvm-readelf")),
                    reason="libsdrgpu.so not built or ROCm LLVM tools absent")
def test_recurrence_kernels_own_their_simd(tmp_path):
    regs = kernel_registers(tmp_path)
    assert len(regs) > 50, "kernel metadata not found"
    own = {k: v for k, v in regs.items()
           if re.search(r"pll_kernel|pll_split_kernel|biquad_kernel", k)}
    assert len(own) >= 20, sorted(own)
    small = {k: v for k, v in own.items() if max(v[0], v[0] + v[1] if v[0] <= 256 else 0) < 512}
    assert not small, f"kernels that leave room on their SIMD: {small}"
    # and the MFMA FIR kernels do not (two waves per SIMD by design)
    fir = [v for k, v in regs.items() if "fir_mxh_kernel" in k]
    assert fir and all(v[0] <= 256 for v in fir)
