"""CPU test: the device libm restatement (csrc/libm_glibc.h) is bit-identical to this host's
glibc sinf / cosf (exhaustive over the PLL's argument range) and atan2f (random pairs).
This is what lets the GPU PLL reproduce the reference's chaotic loop exactly."""
import os
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.parametrize("fma", [0, 1])
def test_libm_restatement_bit_exact(tmp_path, fma):
    exe = tmp_path / f"libm_check{fma}"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-mfma", "-fno-builtin", f"-DSDR_LIBM_FMA={fma}",
                    "-I", os.path.join(ROOT, "unnamed-rust-sdr_amd", "csrc"),
                    os.path.join(ROOT, "tests", "libm_check.c"), "-o", str(exe), "-lm", "-lpthread"],
                   check=True)
    # |x| < 2 pi covers every PLL phase 2 pi * fract(.) ; 40M random atan2f pairs
    r = subprocess.run([str(exe), "6.2832", "40000000"], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
