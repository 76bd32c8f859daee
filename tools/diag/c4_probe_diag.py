"""configs[3] chain probe (round 5): run bank block 1, then PLL block 1 (split kernel, probe
build) beside bank block 2 on another stream, and read back what the PLL's two waves saw.

For every channel the oracle disagrees with, classify each wrong sample by comparing the
helper wave's read-back (c.re, phasedif) with wave 0's shadow of what it wrote:
  stale  : read-back equals the shadow of the same ring slot one or more chunks earlier
  equal  : read-back equals the shadow (the hand-off was right; wave 0's chain itself differs)
  other  : neither
and print the hardware placement (XCC / SE / CU, LDS base and size) of every PLL workgroup and
of the bank workgroups on the same CU.
Run: python tools/experiments/run_with_lib.py LIB.so tools/diag/c4_probe_diag.py [cut]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [os.path.join(ROOT, "unnamed-rust-sdr_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import pyoracle as oracle  # noqa: E402
import scipy.signal as ss  # noqa: E402
import sdrgpu  # noqa: E402
from sdrgpu import _lib  # noqa: E402
from sdrgpu.device import DeviceBuffer  # noqa: E402
from test_pll_gpu import RATE, fm_channels, main_rs_design, oracle_params  # noqa: E402

L = _lib.lib()
KS = 1024
nch, n = 1024, 9000
cut = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
L.sdrgpu_probe_fetch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
L.sdrgpu_probe_bank_fetch.argtypes = [ctypes.c_void_p, ctypes.c_size_t]


def fetch(which, dtype, count):
    a = np.empty(count, dtype)
    assert L.sdrgpu_probe_fetch(which, a.ctypes.data, a.nbytes) == 0
    return a


def hwdec(hwid, lds, xcc):
    # gfx9 HW_ID: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13] tg[19:16] vm[23:20] queue[26:24] state[29:27] me[31:30]
    # LDS_ALLOC: lds_base[7:0] (x 256 B? granularity), lds_size[20:12]
    return dict(xcc=int(xcc) & 0xF, se=(hwid >> 13) & 7, sh=(hwid >> 12) & 1, cu=(hwid >> 8) & 15,
                simd=(hwid >> 4) & 3, wave=hwid & 15, lds_base=lds & 0xFF, lds_size=(lds >> 12) & 0x1FF,
                lds_raw=hex(int(lds)))


rng = np.random.default_rng(45 + nch)
x = fm_channels(rng, nch, n)
taps = ss.firwin(255, 0.2).astype(np.float32)
b = sdrgpu.filter.FirBank(taps, nch, sample_kind=1)
pll = main_rs_design(sdrgpu).design(RATE, nch=nch)
dx = DeviceBuffer.from_numpy(x)
dy = DeviceBuffer.empty(nch * n, np.complex64)
dy.fill_zero()
do = DeviceBuffer.empty(nch * n, np.float32)
dl = DeviceBuffer.empty(nch * n + 8, np.uint8)
assert b.process_dev(dx.ptr, n, cut, dy.ptr, n) == cut
b.sync()
for w in (0, 1):
    assert L.sdrgpu_probe_fetch(w, None, 1024 * KS * 8) == 0
assert L.sdrgpu_probe_fetch(2, None, 64 * 2 * 4 * 8) == 0
rc_bank = L.sdrgpu_probe_bank_fetch(None, 1024 * 4 * 8)
print('bank probe reset rc', rc_bank)
y1 = dy.download().reshape(nch, n)
pll.process_dev(dy.ptr, n, cut, do.ptr, dl.ptr, n)
assert b.process_dev(dx.ptr + 8 * cut, n, n - cut, dy.ptr + 8 * cut, n) == n - cut
b.sync()
pll.sync()
y2 = dy.download().reshape(nch, n)
print("dy[:, :cut] changed during the chain:", int((y1[:, :cut] != y2[:, :cut]).sum()))
out = do.download(dtype=np.float32).reshape(nch, n)[:, :cut]
lk = dl.download(dtype=np.uint8)[:nch * n].reshape(nch, n)[:, :cut]
ro, rl = oracle.pll_batch(oracle_params(oracle), np.ascontiguousarray(y1[:, :cut]), nthreads=16)
bad = (out != ro) | (lk != rl)
chs = np.unique(np.nonzero(bad)[0])
print("GPU PLL vs oracle:", int(bad.sum()), "samples in", chs.size, "channels:", chs.tolist()[:80])

sh = fetch(0, np.complex64, 1024 * KS).reshape(1024, KS)   # (c.re, phasedif) as (re, im)
rb = fetch(1, np.complex64, 1024 * KS).reshape(1024, KS)
hw = fetch(2, np.uint64, 64 * 2 * 4).reshape(64, 2, 4)
bhw = np.empty(1024 * 4, np.uint64)
if rc_bank != 0 or L.sdrgpu_probe_bank_fetch(bhw.ctypes.data, bhw.nbytes) != 0:
    bhw[:] = 0
bhw = bhw.reshape(1024, 4)

m = min(cut, KS)
eq = (sh[:, :m].view(np.uint64) == rb[:, :m].view(np.uint64))
print("hand-off: read-back == shadow in", int(eq.sum()), "of", eq.size, "samples;",
      "mismatching channels:", np.unique(np.nonzero(~eq)[0]).tolist()[:80])
stats = {"stale1": 0, "stale_k": 0, "other": 0}
shu = sh[:, :m].view(np.uint64)
rbu = rb[:, :m].view(np.uint64)
shown = 0
for c in np.unique(np.nonzero(~eq)[0]):
    for s in np.nonzero(~eq[c])[0]:
        hit = None
        for back in range(1, 8):
            sp = s - 16 * back
            if sp < 0:
                break
            if rbu[c, s] == shu[c, sp]:
                hit = back
                break
        if hit == 1:
            stats["stale1"] += 1
        elif hit:
            stats["stale_k"] += 1
        else:
            stats["other"] += 1
        if shown < 12:
            shown += 1
            print(f"  ch {c} s {s} (chunk {s // 8}, k {s % 8}): read {rb[c, s]} shadow {sh[c, s]}"
                  f" shadow[s-16] {sh[c, s - 16] if s >= 16 else None} -> stale by {hit} x 2 chunks")
print("mismatch classes:", stats)
# does the shadow (wave 0's chain) agree with the oracle where the oracle is locked?
locked = rl[:, :m].astype(bool)
chain_ok = (sh[:, :m].imag * np.float32(RATE) == ro[:, :m]) | ~locked
print("wave 0 chain (phasedif * rate) vs oracle output where locked: mismatching samples",
      int((~chain_ok).sum()), "channels", np.unique(np.nonzero(~chain_ok)[0]).tolist()[:40])
# channels by lane group
if chs.size:
    print("bad channels by lane:", np.bincount(chs % 64, minlength=64).tolist())
print("PLL workgroups (xcc se sh cu simd wave lds_base lds_size / t0 t1):")
nblk = nch // 64
for blk in range(nblk):
    for w in range(2):
        r = hw[blk, w]
        d = hwdec(int(r[0]), int(r[1]), int(r[2]))
        t1 = int(r[2]) >> 8
        flag = "BAD" if np.any((chs // 64) == blk) else ""
        print(f"  blk {blk:2d} w{w} xcc {d['xcc']} se {d['se']} sh {d['sh']} cu {d['cu']:2d} simd {d['simd']} "
              f"wave {d['wave']:2d} lds {d['lds_raw']} t0 {int(r[3])} t1 {t1} {flag}")
print("bank workgroups on the same (xcc, se, sh, cu) as each PLL workgroup:")
bank_used = [i for i in range(1024) if bhw[i, 3] != 0]
bd = {i: hwdec(int(bhw[i, 0]), int(bhw[i, 1]), int(bhw[i, 2])) for i in bank_used}
for blk in range(nblk):
    d = hwdec(int(hw[blk, 0, 0]), int(hw[blk, 0, 1]), int(hw[blk, 0, 2]))
    key = (d["xcc"], d["se"], d["sh"], d["cu"])
    co = [i for i in bank_used if (bd[i]["xcc"], bd[i]["se"], bd[i]["sh"], bd[i]["cu"]) == key]
    desc = [(i, bd[i]["lds_raw"], int(bhw[i, 3]), int(bhw[i, 2]) >> 8) for i in co]
    flag = "BAD" if np.any((chs // 64) == blk) else ""
    print(f"  PLL blk {blk:2d} {key} pll lds {d['lds_raw']} t0 {int(hw[blk, 0, 3])}: bank {desc} {flag}")
print("bank workgroups recorded:", len(bank_used))
