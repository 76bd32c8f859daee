#!/bin/bash
# Write round 4's ONE FIR build (the hazard reproducer of DESIGN.md 3.6: its D = 1 bank at 201
# VGPRs lets a 96-VGPR PLL wave share a SIMD) to $1: the round-4 fir_mxh.hip (commit e97e84c)
# with tools/experiments/fir_mxh_one.patch applied.  Needs the git history (build host only).
set -e
cd "$(dirname "$0")/../.."
git show e97e84c:unnamed-rust-sdr_amd/csrc/fir_mxh.hip > "$1"
patch -s "$1" tools/experiments/fir_mxh_one.patch
