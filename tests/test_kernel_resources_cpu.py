"""CPU check of the shipped code object (no GPU): no wave of another kernel can share a SIMD with
the MFMA FIR waves or with the recurrence kernels.  Round 5 measured wrong PLL results (lanes 48-63
of a packed-f32 mixer) when two MFMA bank waves shared the chain wave's SIMD; round 6 traced the
instruction pair (profiles/r06_hazard.txt).  Both sides claim the register file:
  * the PLL and biquad kernels -- serial, split, and the time-parallel seg / refix / fix kernels
    that configs[3] and main.rs run by default -- and the one-wave bf16x3 FIR (fir_mx_kernel)
    allocate all 512 VGPRs (incl. AGPRs) of their SIMD;
  * the two-waves-per-SIMD MFMA FIR kernels (fir_mxh_kernel, fir_mxi_kernel) allocate 256 VGPRs
    and no AGPRs each, so the pair fills the SIMD.
And the two-wave MFMA kernels themselves carry no packed-f32 result read by the next instruction
without a wait state (the same fault inside fir_mxh, round 6: profiles/r06_pkfault.txt).
Reads the amdhsa kernel metadata and disassembly of libsdrgpu.so's gfx950 code objects with the
ROCm LLVM tools."""
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


NEEDS_LIB = pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(f"{LLVM}/llvm-readelf")),
                               reason="libsdrgpu.so not built or ROCm LLVM tools absent")
RECURRENCE = re.compile(r"(pll_kernel|pll_split_kernel|pll_seg_kernel|pll_refix_kernel|pll_fix_kernel|"
                        r"biquad_kernel|bq_seg_kernel|bq_refix_kernel|bq_fix_kernel)I")


@NEEDS_LIB
def test_recurrence_kernels_own_their_simd(tmp_path):
    regs = kernel_registers(tmp_path)
    assert len(regs) > 50, "kernel metadata not found"
    own = {k: v for k, v in regs.items() if RECURRENCE.search(k)}
    # every family and instantiation: 8 PLL designs x (serial x2, split, seg x2, refix x2, fix x2)
    # minus the split kernel's LDS-free variant axis, and 2 x 4 biquad kernels
    for fam in ("pll_kernel", "pll_split_kernel", "pll_seg_kernel", "pll_refix_kernel",
                "pll_fix_kernel", "biquad_kernel", "bq_seg_kernel", "bq_refix_kernel", "bq_fix_kernel"):
        assert any(fam + "I" in k for k in own), f"{fam} not found in the code object"
    assert len(own) >= 70, sorted(own)
    small = {k: v for k, v in own.items() if v[0] < 512}
    assert not small, f"recurrence kernels that leave room on their SIMD: {small}"


@NEEDS_LIB
def test_mfma_fir_kernels_fill_their_simd(tmp_path):
    regs = kernel_registers(tmp_path)
    pair = {k: v for k, v in regs.items() if re.search(r"(fir_mxh_kernel|fir_mxi_kernel)I", k)}
    one = {k: v for k, v in regs.items() if "fir_mx_kernelI" in k}
    assert len(pair) >= 14 and len(one) >= 6, (sorted(pair), sorted(one))
    # two waves per SIMD (waves_per_eu(2, 2), 512-lane workgroups): 256 VGPRs and no AGPRs each
    bad = {k: v for k, v in pair.items() if v != (256, 0)}
    assert not bad, f"two-wave MFMA FIR kernels that leave room on their SIMD: {bad}"
    bad = {k: v for k, v in one.items() if v[0] < 512}
    assert not bad, f"one-wave MFMA FIR kernels that leave room on their SIMD: {bad}"


def code_objects(tmp_path):
    """Paths of the gfx950 code objects bundled in libsdrgpu.so's .hip_fatbin."""
    sec = tmp_path / "fatbin2"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={sec}", LIB,
                    str(tmp_path / "copy2.so")], check=True)
    data = sec.read_bytes()
    out, pos = [], 0
    while (i := data.find(MAGIC, pos)) >= 0:
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple and size:
                co = tmp_path / f"co{len(out)}.o"
                co.write_bytes(data[i + off:i + off + size])
                out.append(co)
        pos = i + len(MAGIC)
    return out


@NEEDS_LIB
def test_two_wave_mfma_kernels_have_no_uncovered_packed_f32_pairs(tmp_path):
    """a v_pk_*_f32 result read by the very next VALU instruction with no wait
    state in between (the compiler leaves none when the producer's op_sel_hi[0] is 0) came out
    wrong in lanes 48-63 while another wave's MFMAs ran on the SIMD -- in the PLL beside bank
    waves, and in fir_mxh's own inf / NaN sums beside its partner wave.  The MFMA FIR kernels
    (fir_mxh and fir_mxi, two waves per SIMD; fir_mx) must contain no such pair, covered (an
    s_nop between) or not."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools", "diag"))
    import pk_hazard_edit as pk
    lines, names = [], []
    for co in code_objects(tmp_path):
        blob = co.read_bytes()
        if b"fir_mxh_kernel" not in blob and b"fir_mxi_kernel" not in blob and b"fir_mx_kernel" not in blob:
            continue  # only the translation units that hold the MFMA FIR kernels
        syms = sorted(set(re.findall(rb"_ZN6sdrgpu12_GLOBAL__N_11[34]fir_mx[hi]?_kernelI\w+", blob)))
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn",
                              "--disassemble-symbols=" + ",".join(x.decode() for x in syms), str(co)],
                             capture_output=True, text=True, check=True).stdout
        cur = None
        for raw in dis.split("\n"):
            m = re.match(r"^[0-9a-f]+ <(\S+)>:", raw)
            if m:
                cur = m.group(1)
                lines.append(cur + ":")
                names.append(cur)
                continue
            lines.append(raw.split("//")[0].rstrip())
            names.append(cur)
    pairs = pk.pairs(lines)
    two_wave = re.compile(r"(fir_mxh_kernel|fir_mxi_kernel|fir_mx_kernel)I")
    seen = {n for n in names if n and two_wave.search(n)}
    assert len(seen) >= 20, sorted(seen)
    uncovered = [(names[a], lines[a].strip()) for a, _, cov, _ in pairs
                 if not cov and names[a] and two_wave.search(names[a])]
    assert not uncovered, f"uncovered packed-f32 pairs in MFMA FIR kernels: {uncovered[:4]}"
    covered = [names[a] for a, _, cov, _ in pairs if cov and names[a] and two_wave.search(names[a])]
    # none either: fir_mxi's digit combination (its 14 covered pairs until round 6) is VOP3 now
    assert not covered, covered
