#!/bin/bash
# Ablated copies of the 64 Ki four-step (fft.hip: fft64k_pass_a / fft64k_pass_b) into
# tools/experiments/abl/ (never the product library), to price configs[2]'s byte stream:
# noflop = both passes keep every load, LDS transpose and store but do no DFT16 / twiddle
# arithmetic (wrong outputs).  Run: python tools/experiments/run_with_lib.py
# tools/experiments/abl/libf64_<v>.so bench_configs.py --config c3 --no-check
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/experiments/abl
make -C unnamed-rust-sdr_amd -s
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v "/fft.o")
for v in ${VARIANTS:-noflop}; do
  src=tools/experiments/abl/fft_$v.hip
  cp unnamed-rust-sdr_amd/csrc/fft.hip $src
  python3 - $src $v <<'PY'
import sys
p, v = sys.argv[1], sys.argv[2]; s = open(p).read()
a = s.index("void fft64k_pass_a(F64Args a) {")
b = s.index("// -------- one-pass radix-4 DIF", a)
body = s[a:b]
if v == "noflop":
    for old in ("Dft<16, false>::run(v);", "if (j) twiddle<16, false>(v, a.tw, 16 * j);",
                "twiddle<16, false>(v, a.tw, col);"):
        assert old in body, old
        body = body.replace(old, "")
    old = "for (int kb = 0; kb < 16; ++kb) v[kb] = cmul(v[kb], w1);"
    assert old in body
    body = body.replace(old, "for (int kb = 0; kb < 16; ++kb) v[kb].x += w1.x;")
s = s[:a] + body + s[b:]
open(p, 'w').write(s)
PY
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -Iunnamed-rust-sdr_amd/csrc -Iinclude -x hip -c $src -o tools/experiments/abl/fft_$v.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/experiments/abl/libf64_$v.so $OBJS tools/experiments/abl/fft_$v.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
echo built
