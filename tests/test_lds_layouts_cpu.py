"""Host restatement of the LDS layouts of the MFMA FIR kernels, checked on the CPU:
every fragment read a wave issues lands on the window sample the GEMM needs, every staged
sample is written where it is read back, and each 16-lane group of a ds_read_b128 (the groups
{0-3,12-15,20-27} / {4-11,16-19,28-31} and their +32 twins) and each 32-lane ds_write_b64 or
64-lane ds_write_b32 hits distinct LDS banks (four-byte banks, 64 of them).

The formulas mirror unnamed-rust-sdr_amd/csrc/fir_mxi.hip (int8 u8 kernel: win_addr<D>, rb[c],
staging at H + 512 k + 8 lane) and fir_mxh.hip at D = 2 (wb0 / hist_addr / new_addr, rb[c])."""
import pytest

READ_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
READ_GROUPS += [[l + 32 for l in g] for g in READ_GROUPS]


def conflict_free_b128(addrs):
    """16-byte reads: distinct addresses must fall in distinct 16-byte bank quads (mod 256 B)."""
    quads = {}
    for a in set(addrs):
        q = (a // 16) % 16
        if q in quads:
            return False
        quads[q] = a
    return True


# ---------------------------------------------------------------- int8 u8 kernel (fir_mxi.hip)
def mxi_win_addr(D, b):
    if D in (1, 2):
        return b
    if D == 8:
        return (b & ~255) | ((((b >> 4) & 15) ^ (2 * ((b >> 8) & 3))) << 4) | (b & 15)
    return 64 * (b >> 6) + 16 * (((b >> 4) & 3) ^ ((b >> 7) & 3)) + (b & 15)


def mxi_geometry(D, NC):
    HR = 64 * NC - 16 * D
    H = (HR + 63) // 64 * 64
    CS = {1: 4, 2: 2, 4: 1, 8: 1}[D]
    return HR, H, H - HR, 256 * D * CS, CS


def mxi_rb(D, NC, v, g, c, OFF):
    if D == 4:
        r = v + c
        return 64 * r + 16 * (g ^ ((r >> 1) & 3))
    return mxi_win_addr(D, OFF + 16 * D * v + 64 * c + 16 * g)


@pytest.mark.parametrize("D,NC", [(4, 3), (4, 5), (2, 3), (2, 5), (1, 3), (1, 5), (8, 4), (8, 6)])
def test_mxi_layout_reads_what_was_staged_conflict_free(D, NC):
    HR, H, OFF, TI, CS = mxi_geometry(D, NC)
    HL = 64 - H // 8
    written = {}
    for lane in range(64):            # staging: 8 samples per lane per group (ds_write_b64)
        if lane >= HL:
            for e in range(8):
                written[8 * (lane - HL) + e] = mxi_win_addr(D, 8 * (lane - HL)) + e
        for k in range(TI // 512):
            s = H + 512 * k + 8 * lane
            for e in range(8):
                written[s + e] = mxi_win_addr(D, s) + e
    assert sorted(written) == list(range(H + TI))
    assert len(set(written.values())) == H + TI and max(written.values()) < H + TI
    for k in range(TI // 512):        # each 32-lane ds_write_b64 pass covers 64 distinct banks
        for half in (range(32), range(32, 64)):
            banks = [((mxi_win_addr(D, H + 512 * k + 8 * l) // 4) + w) % 64 for l in half for w in (0, 1)]
            assert len(set(banks)) == 64
    for j in range(CS):               # fragment reads: lane (v, g) of chunk c, column set j
        for c in range(NC):
            for grp in READ_GROUPS:
                addrs = []
                for l in grp:
                    v, g = l & 15, l >> 4
                    a = mxi_rb(D, NC, v, g, c, OFF) + 256 * D * j
                    p = OFF + 16 * D * v + 64 * c + 16 * g + 256 * D * j
                    assert [written[p + e] for e in range(16)] == list(range(a, a + 16))
                    addrs.append(a)
                assert conflict_free_b128(addrs), (D, NC, j, c, grp[:4])


# ------------------------------------------------ fp16 x 2 kernel at D = 2 (fir_mxh.hip)
def mxh2_wb0(lane):
    return 64 * (lane >> 4) + 4 * (lane & 3) + 16 * (((lane >> 2) & 3) ^ (lane >> 5))


@pytest.mark.parametrize("NCH", [5, 9])
def test_mxh_d2_layout_reads_what_was_staged_conflict_free(NCH):
    D, CS = 2, 2
    HR = 32 * NCH - 16 * D
    H = (HR + 127) // 128 * 128
    assert H == HR
    NH, NG = H // 128, 256 * D * CS // 128
    written = {}
    for lane in range(64):            # one sample pair (4 bytes) per lane per 128-sample group
        for k in range(NH):
            a = (mxh2_wb0(lane) ^ (32 * (k & 1))) + 256 * k
            written[128 * k + 2 * lane], written[128 * k + 2 * lane + 1] = a, a + 2
        for k in range(NG):
            a = (mxh2_wb0(lane) ^ (32 * ((NH + k) & 1))) + 2 * H + 256 * k
            written[H + 128 * k + 2 * lane], written[H + 128 * k + 2 * lane + 1] = a, a + 2
    for k in range(NH + NG):          # every ds_write_b32 wave covers 64 distinct banks
        grp = range(128 * k, 128 * k + 128, 2)
        assert len({(written[s] // 4) % 64 for s in grp}) == 64
    for j in range(CS):
        for c in range(NCH):
            for grp in READ_GROUPS:
                addrs = []
                for l in grp:
                    v, g = l & 15, l >> 4
                    r = v + c
                    a = 64 * r + 16 * (g ^ ((r >> 1) & 3)) + 2 * 256 * D * j
                    p = 32 * v + 32 * c + 8 * g + 256 * D * j
                    assert [written[p + e] for e in range(8)] == list(range(a, a + 16, 2))
                    addrs.append(a)
                assert conflict_free_b128(addrs), (NCH, j, c, grp[:4])


def mxh_layout(D, NCH, CS):
    """fir_mxh.hip's GeoH + staging address functions (byte offsets in one plane of a wave's
    ring, relative to the window start), as in the kernel."""
    TO = 256 * CS
    TI = TO * D
    HR = 32 * NCH - 16 * D
    H = (HR + 127) // 128 * 128

    def wb0(lane):
        if D == 4:
            return 128 * (lane >> 5) + 4 * (lane & 3) + 16 * ((lane >> 2) & 7)
        if D == 2:
            return 64 * (lane >> 4) + 4 * (lane & 3) + 16 * (((lane >> 2) & 3) ^ (lane >> 5))
        return 4 * lane

    def hist_addr(k, lane):
        if D == 4:
            return (wb0(lane) ^ (16 * (k & 7))) + 256 * k
        if D == 2:
            return (wb0(lane) ^ (32 * (k & 1))) + 256 * k
        return wb0(lane) + 256 * k

    def new_addr(k, lane):
        if D == 4:
            return (wb0(lane) ^ (16 * ((H // 128 + k) & 7))) + 128 * (H // 64 + 2 * k)
        if D == 2:
            return (wb0(lane) ^ (32 * ((H // 128 + k) & 1))) + 2 * H + 256 * k
        return wb0(lane) + 2 * H + 256 * k

    return TI, H, hist_addr, new_addr


@pytest.mark.parametrize("D,NCH,CS", [(4, 10, 1), (4, 6, 1), (2, 9, 2), (2, 5, 2), (1, 9, 3), (1, 5, 3), (1, 9, 4), (1, 5, 4)])
def test_mxh_ring_odd_history_is_the_even_windows_tail(D, NCH, CS):
    """fir_mxh.hip's LDS ring (R = H + 2 TI samples; even tiles' window at 0, odd tiles' at TI):
    the bytes where an even window's staging puts its last H new samples are exactly where an
    odd window's history staging (hist_addr, relative to the odd window) would put them, so an
    odd tile that continues the run reads its history in place.  The even history [0, H) and
    the odd window [TI, R) are disjoint, and the ring holds both windows."""
    TI, H, hist_addr, new_addr = mxh_layout(D, NCH, CS)
    NG, NH = TI // 128, H // 128
    R = H + 2 * TI
    WODD = 2 * TI                                    # bytes: TI samples x 2 B per plane
    even = {}                                        # window sample -> byte (even window)
    for k in range(NG):
        for lane in range(64):
            a = new_addr(k, lane)
            even[H + 128 * k + 2 * lane] = a
    for k in range(NH):                              # odd history sample s (odd-relative)
        for lane in range(64):
            s = 128 * k + 2 * lane
            assert WODD + hist_addr(k, lane) == even[TI + s], (k, lane)
    assert TI >= H
    top = max(max(new_addr(k, l) for k in range(NG) for l in range(64)), 0) + 4
    assert top <= 2 * (H + TI) and WODD + top <= 2 * R      # both windows inside the ring
