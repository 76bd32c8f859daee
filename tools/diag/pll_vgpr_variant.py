"""Copy of pll.hip with a VGPR cap on the split and/or the LDS-free PLL kernel (round 5 chain
discriminator: does the configs[3] mismatch need the LDS ring, or only a PLL wave sharing a SIMD
whose register file two bank waves nearly fill?).  Diagnostic only.

  python tools/diag/pll_vgpr_variant.py OUT SPLIT_CAP SCALAR_CAP ROUTE
  [excl]: reserve 512 VGPRs per PLL wave (one wave per SIMD)
  SPLIT_CAP / SCALAR_CAP: min waves per SIMD (VGPRs <= 512 / w, granule 8; 0 = unchanged); ROUTE: split | scalar (main.rs launches)
"""
import sys

out, split_cap, scalar_cap, route = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
excl = len(sys.argv) > 5 and sys.argv[5] == "excl"  # reserve the whole register file (v255 + a255)
s = open("unnamed-rust-sdr_amd/csrc/pll.hip").read()
if excl:
    for old in ("    const long ch = (long)blockIdx.x * kPllBlock + threadIdx.x;\n    if (ch >= p.nch) return;\n",
                "    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;\n"):
        assert s.count(old) == 1, old
        s = s.replace(old, '    asm volatile("" ::: "v255", "a255");\n' + old)
old = "__global__ __launch_bounds__(kPllBlock) void pll_kernel("
assert s.count(old) == 1
if scalar_cap:
    s = s.replace(old, f"__global__ __launch_bounds__(kPllBlock) __attribute__((amdgpu_waves_per_eu({scalar_cap}))) void pll_kernel(")
old = "__global__ __launch_bounds__(2 * kPllBlock) void pll_split_kernel("
assert s.count(old) == 1
if split_cap:
    s = s.replace(old, f"__global__ __launch_bounds__(2 * kPllBlock) __attribute__((amdgpu_waves_per_eu({split_cap}))) void pll_split_kernel(")
old = "    if (vec && (MODE == 0 || MODE == 1))"
assert s.count(old) == 1
if route == "scalar":
    s = s.replace(old, "    if (false && vec && (MODE == 0 || MODE == 1))")
else:
    assert route == "split"
open(out, "w").write(s)
