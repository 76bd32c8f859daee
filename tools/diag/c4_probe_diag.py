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
assert L.sdrgpu_probe_fetch(0, None, 1024 * KS * 16) == 0
assert L.sdrgpu_probe_fetch(1, None, 1024 * KS * 8) == 0
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

sh4 = fetch(0, np.float32, 1024 * KS * 4).reshape(1024, KS, 4)  # (v.re, v.im, c.re, c.im)
sh_vr, sh_vi, sh_cr, sh_ci = (sh4[:, :, q] for q in range(4))
rb = fetch(1, np.complex64, 1024 * KS).reshape(1024, KS)   # (c.re, phasedif) the helper read
sh = rb.copy()  # ring contents as read back (the hand-off was verified equal to wave 0's values)
sh.real = sh_cr
hw = fetch(2, np.uint64, 64 * 2 * 4).reshape(64, 2, 4)
bhw = np.empty(1024 * 4, np.uint64)
if rc_bank != 0 or L.sdrgpu_probe_bank_fetch(bhw.ctypes.data, bhw.nbytes) != 0:
    bhw[:] = 0
bhw = bhw.reshape(1024, 4)

m = min(cut, KS)
have_shadow = not np.all(sh4.view(np.uint32) == np.uint32(0xFFFFFFFF))
if have_shadow:
    eq = (sh[:, :m].view(np.uint64) == rb[:, :m].view(np.uint64))
    print("hand-off: read-back == shadow in", int(eq.sum()), "of", eq.size, "samples;",
          "mismatching channels:", np.unique(np.nonzero(~eq)[0]).tolist()[:80])
    stats = {"stale1": 0, "stale_k": 0, "other": 0}
    shu = sh[:, :m].view(np.uint64)
    rbu = rb[:, :m].view(np.uint64)
    shown = 0
    for c in np.unique(np.nonzero(~eq)[0]):
        for s_ in np.nonzero(~eq[c])[0]:
            hit = None
            for back in range(1, 8):
                sp = s_ - 16 * back
                if sp < 0:
                    break
                if rbu[c, s_] == shu[c, sp]:
                    hit = back
                    break
            stats["stale1" if hit == 1 else ("stale_k" if hit else "other")] += 1
            if shown < 12:
                shown += 1
                print(f"  ch {c} s {s_} (chunk {s_ // 8}, k {s_ % 8}): read {rb[c, s_]} shadow {sh[c, s_]}"
                      f" shadow[s-16] {sh[c, s_ - 16] if s_ >= 16 else None} -> stale by {hit} x 2 chunks")
    print("mismatch classes:", stats)
# does the shadow (wave 0's chain) agree with the oracle where the oracle is locked?
if have_shadow:
    locked = rl[:, :m].astype(bool)
    chain_ok = (sh[:, :m].imag * np.float32(RATE) == ro[:, :m]) | ~locked
    print("wave 0 chain (phasedif * rate) vs oracle output where locked: mismatching samples",
          int((~chain_ok).sum()), "channels", np.unique(np.nonzero(~chain_ok)[0]).tolist()[:40])
# wave 0's inputs vs the snapshot, and a step-by-step restatement of its chain (pll.rs:71-76 in
# f32 with glibc atan2f / sincosf) from the snapshot: where does wave 0 first differ, and in what?
if have_shadow and chs.size:
    m2 = min(cut, KS)
    xin = y1[:, :m2]
    cc = chs[:64]
    f32 = np.float32
    b0, b1, b2, na1, na2 = [f32(v) for v in oracle.biquad_coefs(1, 80000.0, 0.7, RATE)]
    gain = f32(0.035)
    refc = f32(0.0) / f32(RATE)
    two_pi = f32(2.0) * f32(3.14159265358979323846)
    z = lambda: np.zeros(cc.size, f32)
    vr, vi, nph = z(), z(), z()
    lx1r, lx2r, ly1r, ly2r, lx1i, lx2i, ly1i, ly2i = (z() for _ in range(8))
    first = np.full(cc.size, -1)
    what = [""] * cc.size
    for i in range(m2):
        x = xin[cc, i]
        xr, xi = x.real.astype(f32), x.imag.astype(f32)
        cjr, cji = vr, -vi
        cr = xr * cjr - xi * cji
        ci = xr * cji + xi * cjr
        orr = f32(0) + cr * b0; oi = f32(0) + ci * b0
        orr = orr + lx1r * b1; oi = oi + lx1i * b1
        orr = orr + lx2r * b2; oi = oi + lx2i * b2
        orr = orr + ly1r * na1; oi = oi + ly1i * na1
        orr = orr + ly2r * na2; oi = oi + ly2i * na2
        lx2r, lx1r, ly2r, ly1r = lx1r, cr, ly1r, orr
        lx2i, lx1i, ly2i, ly1i = lx1i, ci, ly1i, oi
        pd = oracle.atan2f(oi, orr) * gain
        nph = nph + (refc + pd)
        nph = nph - np.trunc(nph)
        sn, cs = oracle.sincosf(two_pi * nph)
        vr, vi = f32(1.0) * cs, f32(1.0) * sn
        gcr, gci, gvr, gvi = sh_cr[cc, i], sh_ci[cc, i], sh_vr[cc, i], sh_vi[cc, i]
        gpd = rb[cc, i].imag
        for j in np.nonzero((first < 0) & ((gcr != cr) | (gci != ci) | (gvr != vr) | (gvi != vi) | (gpd != pd)))[0]:
            first[j] = i
            c_ = cc[j]
            pvr, pvi = (sh_vr[c_, i - 1], sh_vi[c_, i - 1]) if i else (f32(0), f32(0))
            xr_, xi_ = f32(xin[c_, i].real), f32(xin[c_, i].imag)
            ecr = xr_ * pvr - xi_ * (-pvi)
            eci = xr_ * (-pvi) + xi_ * pvr
            what[j] = (f"s {i}: c gpu ({gcr[j]!r}, {gci[j]!r}) emu ({cr[j]!r}, {ci[j]!r}); x * conj(gpu v[s-1]) = ({ecr!r}, {eci!r}) | "
                       f"v gpu ({gvr[j]!r}, {gvi[j]!r}) emu ({vr[j]!r}, {vi[j]!r}) | phasedif gpu {gpd[j]!r} emu {pd[j]!r} | "
                       f"gpu v[s-1] ({pvr!r}, {pvi!r})")
        # continue from the GPU's own values where they diverge?  No: the emulation stays on the
        # reference path, so `first` is the first divergent sample of each channel.
    for j in range(min(cc.size, 24)):
        print(f"  ch {cc[j]} (lane {cc[j] % 64}): first divergence {what[j] or 'none in the probe window'}")
    if os.environ.get("PROBE_NPZ"):
        np.savez_compressed(os.environ["PROBE_NPZ"], chans=cc, x=xin[cc], shadow=sh4[cc], readback=rb[cc],
                            first=first, gpu_out=out[cc, :m2], gpu_lock=lk[cc, :m2], ref_out=ro[cc, :m2],
                            ref_lock=rl[cc, :m2])

# channels by lane group
if chs.size:
    print("bad channels by lane:", np.bincount(chs % 64, minlength=64).tolist())
print("PLL workgroups (xcc se sh cu simd wave lds / start time):")
nblk = nch // 64
for blk in range(nblk):
    for w in range(2):
        r = hw[blk, w]
        if int(r[3]) in (0, 0xFFFFFFFFFFFFFFFF):
            continue
        d = hwdec(int(r[0]), int(r[1]), int(r[2]))
        flag = "BAD" if np.any((chs // 64) == blk) else ""
        print(f"  blk {blk:2d} w{w} xcc {d['xcc']} se {d['se']} sh {d['sh']} cu {d['cu']:2d} simd {d['simd']} "
              f"wave {d['wave']:2d} lds {d['lds_raw']} t0 {int(r[3])} {flag}")
print("bank workgroups on the same (xcc, se, sh, cu) as each PLL workgroup:")
bank_used = [i for i in range(1024) if bhw[i, 3] != 0]
bd = {i: hwdec(int(bhw[i, 0]), int(bhw[i, 1]), int(bhw[i, 2])) for i in bank_used}
for blk in range(nblk):
    d = hwdec(int(hw[blk, 0, 0]), int(hw[blk, 0, 1]), int(hw[blk, 0, 2]))
    key = (d["xcc"], d["se"], d["sh"], d["cu"])
    co = [i for i in bank_used if (bd[i]["xcc"], bd[i]["se"], bd[i]["sh"], bd[i]["cu"]) == key]
    desc = [(i, bd[i]["lds_raw"], "end", int(bhw[i, 3])) for i in co]
    flag = "BAD" if np.any((chs // 64) == blk) else ""
    print(f"  PLL blk {blk:2d} {key} pll lds {d['lds_raw']} t0 {int(hw[blk, 0, 3])}: bank {desc} {flag}")
print("bank workgroups recorded:", len(bank_used))
ncores = sum(1 for blk in range(nblk) if any(
    (bd[i]["xcc"], bd[i]["se"], bd[i]["sh"], bd[i]["cu"]) == (lambda d: (d["xcc"], d["se"], d["sh"], d["cu"]))(
        hwdec(int(hw[blk, 0, 0]), int(hw[blk, 0, 1]), int(hw[blk, 0, 2]))) for i in bank_used))
print(f"SUMMARY: {int(bad.sum())} wrong PLL samples in {chs.size} channels; "
      f"{ncores} of {nblk} PLL workgroups share a CU with a bank workgroup")
