#!/bin/bash
# Ablated copies of the any-N FFT tile kernel (fft_gen.hip) into tools/experiments/abl/
# (never the product library): nofft = no passes (gather + store only), nodb = linear
# value instead of 20 log10 |X| in the dB store, noload = constant samples instead of the
# frame gather.  Run: python tools/experiments/run_with_lib.py tools/experiments/abl/libfg_<v>.so bench_configs.py --config ex
set -e
cd "$(dirname "$0")/../.."
mkdir -p tools/experiments/abl
make -C unnamed-rust-sdr_amd -s
OBJS=$(ls unnamed-rust-sdr_amd/build/*.o | grep -v fft_gen.o)
for v in ${VARIANTS:-nofft nodb noload}; do
  src=tools/experiments/abl/fft_gen_$v.hip
  cp unnamed-rust-sdr_amd/csrc/fft_gen.hip $src
  python3 - $src $v <<'PY'
import sys
p, v = sys.argv[1], sys.argv[2]; s = open(p).read()
if v == "nofft":
    old = "gen_engine<BLK, TILE>(b0, N, B, a.rl, a.tw);"
    assert old in s; s = s.replace(old, "")
elif v == "nodb":
    old = "else reinterpret_cast<float*>(a.out)[(f0 + f) * N + o] = db_of(x, a.norm);"
    assert old in s; s = s.replace(old, "else reinterpret_cast<float*>(a.out)[(f0 + f) * N + o] = x.x * a.norm;")
elif v == "noload":
    old = "gather_tile<PER, BLK>(a.src, N, f0, nf, L, [&](int p) { return a.rl.dn.div(p); }, v);"
    assert old in s
    s = s.replace(old, "for (int u = 0; u < PER; ++u) v[u] = make_float2((float)u, (float)threadIdx.x);")
open(p, 'w').write(s)
PY
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -Iunnamed-rust-sdr_amd/csrc -Iinclude -x hip -c $src -o tools/experiments/abl/fft_gen_$v.o
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/experiments/abl/libfg_$v.so $OBJS tools/experiments/abl/fft_gen_$v.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
echo built
