"""Host-side check of the LDS-DMA piece plans of the wide stride-1 conv
(dlq_amd/csrc/conv3x3i.hip) and the stride-2 conv + fused downsample
(dlq_amd/csrc/conv3x3s2i.hip).  Test infrastructure, not product code.

The kernels' plan and tap addressing are restated here in numpy, index
expression for index expression (the constants of IGeo / JGeo, prep_issue,
issue_piece, the compute side's col_off / mid_off / left_off, make_perm), and
for every shape and batch size asked for it proves:

  * every DMA piece of every stage of every workgroup is issued exactly once
    (over the 8 waves and their DPW piece slots), each of one kind;
  * every source byte is inside its buffer: the NHWC input tensor, the zero
    block (1 KiB; slice j adds 32 j), the packed weight image;
  * every LDS destination lies inside its slot's weight / patch region and
    below the LDS budget; no two pieces of a stage overlap;
  * the tap reads see the right bytes: for every output pixel of every item
    and every 3x3 tap, the LDS unit the MFMA's B fragment reads holds the
    input pixel (n, ih, iw, plane) the reference im2col
    (RK/kernels/im2col.cu:37-54) puts in that K column -- or a zero when the
    tap is padding, and then the unit is a zero unit (zero-block DMA or the
    slot's zero region);
  * the int32 offset arithmetic the kernels do in `int` stays below 2^31
    (the 64-bit pointer sums take it from there: a.x + (size_t)(int offset)),
    which bounds the batch a launch may take; the saddr bases are 64-bit
    pointer arithmetic on the kernel's own pointers, so no base is assembled
    from 32-bit halves (the round-2 sign-extension fault).

With emit= a dict, the two checks also return each wave's LDS-DMA pieces in
issue order -- (LDS address, 64 source codes: kind << 48 | byte offset, kinds
X input, Z zero block, W conv weights, D downsample weights) per (workgroup,
wave) -- which tests/test_gpu_dma_plan.py compares with the pieces the
compiled kernels record in a plan-capture build (tools/check/plan_capture.hip):
the restatement is pinned to the kernels, not only to itself.

Run: python tools/check/dma_plan.py [N ...]   (tests/test_dma_plan.py runs it)
"""
from __future__ import annotations

import sys

import numpy as np

NCU = 256          # CUs (the launchers read the device attribute; 256 on MI355X)
INT_MAX = 2**31 - 1


def xcd_remap(bid, nblk):
    xcd, q, r = bid & 7, nblk >> 3, nblk & 7
    base = xcd * (q + 1) if xcd < r else r * (q + 1) + (xcd - r) * q
    return base + (bid >> 3)


class Fail(AssertionError):
    pass


KX, KZ, KW, KD = 1, 2, 3, 4  # source kinds of emitted pieces


def code(kind, off):
    return (np.int64(kind) << np.int64(48)) | np.asarray(off, dtype=np.int64)


def need(cond, msg):
    if not np.all(cond):
        raise Fail(msg)


# ---------------------------------------------------------------- conv3x3i
def igeo(W, SPS=1):
    IL, ISC, IPITCH = 392, 32, 9 * 32 + 16
    H = W
    RPI = W if W < 14 else 14
    IPI = IL // (RPI * W)
    OT = 64 if W == 7 else 128
    RW = W
    CS0 = (RPI + 2) * RW
    CS = CS0 + (((RPI * W - CS0) % 16) + 16) % 16
    UP = (IPI * CS + 15) // 16 * 16
    PP = (2 * UP + 63) // 64
    ZU = 2 * W + 16
    WB = OT * IPITCH
    WP = WB // 1024
    ZB = (ZU * 16 + 255) // 256 * 256
    WBS, PB = SPS * WB, PP * 1024 + ZB   # slot: [SPS weight blocks][SPS x (patch, zero region)]
    OFF_P = WBS
    OFF_Z = OFF_P + PP * 1024
    SLOT = WBS + SPS * PB
    return dict(IL=IL, ISC=ISC, IPITCH=IPITCH, H=H, RPI=RPI, IPI=IPI, OT=OT, MT=OT // 32, RW=RW, CS=CS, UP=UP,
                PP=PP, ZU=ZU, WB=WB, WP=WP, SPS=SPS, WBS=WBS, PB=PB, OFF_P=OFF_P, PPS=SPS * PP, WPS=SPS * WP,
                NPIECE=SPS * (WP + PP), OFF_Z=OFF_Z, SLOT=SLOT, OFF_AB=2 * SLOT)


def check_conv3x3i(W, N, emit=None):
    C = {28: 128, 14: 256, 7: 512}[W]
    SPS = 2 if W == 7 else 1  # int8: the 7x7 launches take two 32-channel slices per stage (sps_of)
    g = igeo(W, SPS)
    H, IL, OT, NSL, NLD = W, g["IL"], g["OT"], C // 32, 8
    NS = NSL // SPS
    P = N * H * W
    OCp = C
    n_ot, n_pi = OCp // OT, (P + IL - 1) // IL
    NI = n_ot * n_pi
    Gd = min(NI, NCU)
    # WideStream: patch slots k < KPP (piece wv + NLD k), weight slots after
    # (piece wv + NLD (k - KPP)); a wave with no piece at a slot issues it
    # masked (EXEC = 0: nothing is read or written, nothing is recorded)
    KPP = (g["PPS"] + NLD - 1) // NLD
    KPW = (g["WPS"] + NLD - 1) // NLD
    DPW = KPP + KPW
    lds_total = g["OFF_AB"] + 2 * C * 4
    need(lds_total <= 160 * 1024, "LDS budget")
    xbytes = P * C
    wbytes = (OCp // 128 if OCp >= 128 else 1) * NSL * 128 * g["IPITCH"]
    lane = np.arange(64)
    # int32 offset arithmetic of prep_issue: ((n*H+ih)*W+iw)*C + plane*16
    need(P * C < INT_MAX, f"conv3x3i W={W}: N={N} overflows the int pixel offset")
    # units of the patch (slot-relative unit index u -> content)
    u = np.arange(g["PP"] * 64)
    plane = (u >= g["UP"]).astype(int)
    q = u - plane * g["UP"]
    c, rem = q // g["CS"], q % g["CS"]
    r, iw = rem // g["RW"], rem % g["RW"]
    # compute side, per (tile, lane): pixel, taps
    tiles = np.arange(13)
    lp_all = tiles[:, None] * 32 + np.arange(32)[None, :]
    lp = np.minimum(lp_all, IL - 1)
    cc, rr = lp // (g["RPI"] * W), lp % (g["RPI"] * W)
    rrow, ow = rr // W, rr % W
    bu = cc * g["CS"] + rrow * g["RW"] + ow
    for b in range(Gd):
        bb = xcd_remap(b, Gd)
        nst = ((NI - bb + Gd - 1) // Gd) * NS
        for li in range(nst // NS):
            it = bb + li * Gd
            ot, p0 = it % n_ot, (it // n_ot) * IL
            R0 = p0 // W
            gr = R0 + c * g["RPI"]
            n = gr // H
            ih = gr - n * H + r - 1
            ok = (u < 2 * g["UP"]) & (c < g["IPI"]) & (r < g["RPI"] + 2) & (n < N) & (ih >= 0) & (ih < H) & \
                 (iw >= 0) & (iw < W)
            src = np.where(ok, ((n * H + ih) * W + iw) * C + plane * 16, -1)
            o128, ohalf = (ot * OT) >> 7, (ot * OT) & 127
            wbase = (o128 * NSL * 128 + ohalf) * g["IPITCH"]
            for st in range(NS):
                s_idx = li * NS + st  # the workgroup's stage index (slot s_idx % 2)
                j0 = st * SPS  # the stage's first slice
                issued = np.zeros(g["NPIECE"], int)
                for wv in range(NLD):
                    for k in range(DPW):
                        pc = wv + k * NLD if k < KPP else None
                        wp = wv + (k - KPP) * NLD if k >= KPP else None
                        if pc is not None and pc < g["PPS"]:
                            sub = 1 if (SPS > 1 and pc >= g["PP"]) else 0
                            p = pc - sub * g["PP"]
                            j = j0 + sub
                            us = p * 64 + lane
                            s_ok = src[us] >= 0
                            need(src[us][s_ok] + j * 32 + 16 <= xbytes, "patch source past the input")
                            need(src[us][s_ok] + j * 32 >= 0, "patch source before the input")
                            need((lane[~s_ok] & 3) * 16 + j * 32 + 16 <= 1024, "zero source past the zero block")
                            dst = g["OFF_P"] + sub * g["PB"] + p * 1024
                            need(dst + 1024 <= g["OFF_Z"] + sub * g["PB"], "patch piece into the zero region")
                            issued[pc] += 1
                            if emit is not None:
                                emit.setdefault((b, wv), []).append(
                                    (s_idx % 2 * g["SLOT"] + dst,
                                     np.where(s_ok, code(KX, src[us] + j * 32), code(KZ, (lane & 3) * 16 + j * 32))))
                        elif wp is not None and wp < g["WPS"]:
                            sub = 1 if (SPS > 1 and wp >= g["WP"]) else 0
                            q = wp - sub * g["WP"]
                            s0 = wbase + (j0 + sub) * 128 * g["IPITCH"] + q * 1024
                            need(s0 >= 0 and s0 + 1024 <= wbytes, "weight piece past the packed image")
                            need(sub * g["WB"] + q * 1024 + 1024 <= g["WBS"], "weight piece past the weight region")
                            issued[g["PPS"] + wp] += 1
                            if emit is not None:
                                emit.setdefault((b, wv), []).append(
                                    (s_idx % 2 * g["SLOT"] + wp * 1024, code(KW, s0 + 16 * lane)))
                need(issued == 1, f"conv3x3i W={W}: a piece issued {issued.min()}..{issued.max()} times")
            # tap reads of the item: every output pixel, every tap, both planes
            p = p0 + lp_all
            valid = (lp_all < IL) & (p < P)
            pn = p // (H * W)
            poh, pow_ = (p % (H * W)) // W, p % W
            for lh, sub in ((0, 0), (1, 0), (0, SPS - 1), (1, SPS - 1)):
                mid = g["OFF_P"] + lh * g["UP"] * 16 + bu * 16
                zo = g["OFF_Z"] + sub * g["PB"]  # this slice's zero region
                for kh in range(3):
                    for kw in range(3):
                        if kw == 1:
                            addr = mid
                        elif kw == 0:
                            addr = np.where(ow == 0, g["OFF_Z"] + ((bu - 1) & 15) * 16, mid - 16)
                        else:
                            addr = np.where(ow == W - 1, g["OFF_Z"] + ((bu + 1) & 15) * 16, mid + 16)
                        addr = addr + kh * g["RW"] * 16 + sub * g["PB"]  # the kernel's b_off
                        need(addr + 16 <= g["SLOT"], "tap read past the slot")
                        eih, eiw = poh + kh - 1, pow_ + kw - 1
                        inside = (eih >= 0) & (eih < H) & (eiw >= 0) & (eiw < W)
                        in_zero = (addr >= zo) & (addr < zo + g["ZU"] * 16)
                        unit = (addr - g["OFF_P"] - sub * g["PB"]) // 16
                        need((addr % 16 == 0), "unaligned tap read")
                        need(in_zero | ((unit >= 0) & (unit < g["PP"] * 64)), "tap read outside patch and zero region")
                        want = np.where(inside, ((pn * H + eih) * W + eiw) * C + lh * 16, -1)
                        got = np.where(in_zero, -1, src[np.clip(unit, 0, g["PP"] * 64 - 1)])
                        need(~valid | (got == want), f"conv3x3i W={W} N={N}: wrong tap bytes (kh={kh} kw={kw})")


# ---------------------------------------------------------------- conv3x3s2i
def jgeo(OW, DS=True, NSR=0):
    JL, JWP, JDP, JOT = 196, 9 * 32 + 16, 32 + 16, 128
    OH, WI, HI = OW, 2 * OW, 2 * OW
    RPI = OW if OW < 14 else (14 if OW == 14 else 7)
    IPI = JL // (RPI * OW)
    IRC = 2 * RPI + 1
    CS = IRC * WI + (1 if OW == 7 else 0)
    UP = (IPI * CS + 15) // 16 * 16
    PP = (2 * UP + 63) // 64
    WB, DB = JOT * JWP, JOT * JDP
    WP = (WB + (DB if DS else 0)) // 1024
    WPC = 0 if NSR else WP
    W_ALL = NSR * WP * 1024
    OFF_P = W_ALL if NSR else WB + DB
    ZU = 2 * WI + 16
    OFF_Z = OFF_P + PP * 1024
    ZB = (ZU * 16 + 255) // 256 * 256
    SLOT = PP * 1024 + ZB if NSR else OFF_Z + ZB
    OFF_AB = W_ALL + 2 * SLOT if NSR else 2 * SLOT
    return dict(JL=JL, JWP=JWP, JDP=JDP, JOT=JOT, OH=OH, WI=WI, HI=HI, RPI=RPI, IPI=IPI, IRC=IRC, CS=CS, UP=UP, PP=PP,
                WB=WB, DB=DB, WP=WP, WPC=WPC, NPIECE=WPC + PP, W_ALL=W_ALL, OFF_P=OFF_P, ZU=ZU, OFF_Z=OFF_Z, ZB=ZB,
                SLOT=SLOT, OFF_AB=OFF_AB)


def make_perm(OW):
    g = jgeo(OW)
    LA = [0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27]
    LB = [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]
    px = [-1] * (7 * 32)
    cnt, donor = [0] * 16, [-1] * 16
    for p in range(g["JL"]):
        c, rem = p // (g["RPI"] * OW), p % (g["RPI"] * OW)
        r, ow = rem // OW, rem % OW
        q = (c * g["CS"] + 2 * r * g["WI"] + ow) & 15
        k = cnt[q]
        cnt[q] += 1
        if donor[q] < 0:
            donor[q] = p
        px[(k // 2) * 32 + (LB[q] if k & 1 else LA[q])] = p
    for tile in range(7):
        for q in range(16):
            for L in (LA, LB):
                if px[tile * 32 + L[q]] < 0:
                    px[tile * 32 + L[q]] = donor[q] | 0x4000
    return np.array(px)


def check_s2i(OW, N, emit=None):
    C = {28: 64, 14: 128, 7: 256}[OW]
    OC, NS, JNW = 2 * C, C // 32, 8
    RW = OW == 28  # layer2.0: resident weights (OCp == JOT)
    g = jgeo(OW, True, NS if RW else 0)
    HI, WI = g["HI"], g["WI"]
    P = N * OW * OW
    n_ot = OC // g["JOT"]
    NI = n_ot * ((P + g["JL"] - 1) // g["JL"])
    Gd = min(NI, NCU)
    # s2i_body: patch slots k < KPP (piece wv + 8 k), then weight slots
    # (weight piece wv + 8 (k - KPP)); empty slots are issued masked
    KPP = (g["PP"] + JNW - 1) // JNW
    KPW = (g["WPC"] + JNW - 1) // JNW
    DPW = KPP + KPW
    WCP = g["WB"] // 1024
    lds_total = g["OFF_AB"] + 4 * OC * 4
    need(lds_total <= 160 * 1024, "LDS budget")
    xbytes = N * HI * WI * C
    wbytes_c, wbytes_d = n_ot * NS * g["WB"], n_ot * NS * g["DB"]
    need(xbytes < INT_MAX, f"conv3x3s2i OW={OW}: N={N} overflows the int pixel offset")
    lane = np.arange(64)
    rw_pieces = []  # (wave, LDS address, codes) of the resident-weight prologue
    if RW:  # resident weights: every stage's block once, pc = wave + 8 i
        NW = NS * g["WP"]
        for pc in range(NW):
            j, qq = pc // g["WP"], pc % g["WP"]
            if qq < WCP:
                need(j * g["WB"] + qq * 1024 + 1024 <= wbytes_c, "resident conv weight piece past the image")
                cd = code(KW, j * g["WB"] + qq * 1024 + 16 * lane)
            else:
                need(j * g["DB"] + (qq - WCP) * 1024 + 1024 <= wbytes_d, "resident ds weight piece past the image")
                cd = code(KD, j * g["DB"] + (qq - WCP) * 1024 + 16 * lane)
            need(pc * 1024 + 1024 <= g["W_ALL"], "resident weights past their region")
            rw_pieces.append((pc % JNW, pc * 1024, cd))
    u = np.arange(g["PP"] * 64)
    plane = (u >= g["UP"]).astype(int)
    q = u - plane * g["UP"]
    c, rem = q // g["CS"], q % g["CS"]
    r, pos = rem // WI, rem % WI
    iw = np.where(pos < OW, 2 * pos, 2 * (pos - OW) + 1)
    perm = make_perm(OW)
    lp_raw = perm
    lp = lp_raw & 0x3FFF
    real = (lp_raw & 0x4000) == 0
    cc, rr = lp // (g["RPI"] * OW), lp % (g["RPI"] * OW)
    rrow, ow = rr // OW, rr % OW
    bu = cc * g["CS"] + 2 * rrow * WI + ow
    need(np.sort(lp[real]).tolist() == list(range(g["JL"])), "pixel permutation is not a bijection")
    for b in range(Gd):
        bb = xcd_remap(b, Gd)
        nst = ((NI - bb + Gd - 1) // Gd) * NS
        if emit is not None:
            for wv, dst, cd in rw_pieces:
                emit.setdefault((b, wv), []).append((dst, cd))
        for li in range(nst // NS):
            it = bb + li * Gd
            ot, p0 = it % n_ot, (it // n_ot) * g["JL"]
            R0 = p0 // OW
            gr = R0 + c * g["RPI"]
            n = gr // g["OH"]
            ih = 2 * (gr - n * g["OH"]) - 1 + r
            ok = (u < 2 * g["UP"]) & (c < g["IPI"]) & (r < g["IRC"]) & (n < N) & (ih >= 0) & (ih < HI)
            src = np.where(ok, ((n * HI + ih) * WI + iw) * C + plane * 16, -1)
            for j in range(NS):
                s_idx = li * NS + j  # the workgroup's stage index (slot s_idx % 2)
                issued = np.zeros(g["NPIECE"], int)
                for wv in range(JNW):
                    for k in range(DPW):
                        pc = wv + k * JNW if k < KPP else None
                        wp = wv + (k - KPP) * JNW if k >= KPP else None
                        if pc is not None and pc < g["PP"]:
                            us = pc * 64 + lane
                            s_ok = src[us] >= 0
                            need(src[us][s_ok] + j * 32 + 16 <= xbytes, "patch source past the input")
                            need((lane[~s_ok] & 3) * 16 + j * 32 + 16 <= 1024, "zero source past the zero block")
                            need(g["OFF_P"] + pc * 1024 + 1024 <= g["OFF_Z"], "patch piece into the zero region")
                            issued[pc] += 1
                            if emit is not None:
                                emit.setdefault((b, wv), []).append(
                                    (s_idx % 2 * g["SLOT"] + g["OFF_P"] + pc * 1024,
                                     np.where(s_ok, code(KX, src[us] + j * 32), code(KZ, (lane & 3) * 16 + j * 32))))
                        elif wp is not None and wp < g["WPC"]:
                            if wp < WCP:
                                s0 = ot * NS * g["WB"] + j * g["WB"] + wp * 1024
                                need(s0 + 1024 <= wbytes_c, "conv weight piece past the image")
                            else:
                                s0 = ot * NS * g["DB"] + j * g["DB"] + (wp - WCP) * 1024
                                need(s0 + 1024 <= wbytes_d, "ds weight piece past the image")
                            need(wp * 1024 + 1024 <= g["OFF_P"], "weight piece into the patch region")
                            issued[g["PP"] + wp] += 1
                            if emit is not None:
                                emit.setdefault((b, wv), []).append(
                                    (s_idx % 2 * g["SLOT"] + wp * 1024, code(KW if wp < WCP else KD, s0 + 16 * lane)))
                need(issued == 1, f"s2i OW={OW}: a piece issued {issued.min()}..{issued.max()} times")
            p = p0 + lp
            valid = real & (p < P)
            pn = p // (OW * OW)
            poh, pow_ = (p % (OW * OW)) // OW, p % OW
            for lh in (0, 1):
                mid = g["OFF_P"] + lh * g["UP"] * 16 + bu * 16
                left = np.where(ow == 0, g["OFF_Z"] + ((bu + OW - 1) & 15) * 16, mid + (OW - 1) * 16)
                for kh in range(3):
                    for kw in range(3):
                        base = left if kw == 0 else mid
                        addr = base + (kh * WI + (OW if kw == 2 else 0)) * 16
                        eih, eiw = 2 * poh + kh - 1, 2 * pow_ + kw - 1
                        inside = (eih >= 0) & (eih < HI) & (eiw >= 0) & (eiw < WI)
                        in_zero = (addr >= g["OFF_Z"]) & (addr < g["OFF_Z"] + g["ZU"] * 16)
                        unit = (addr - g["OFF_P"]) // 16
                        need(in_zero | ((unit >= 0) & (unit < g["PP"] * 64)), "tap read outside patch and zero region")
                        want = np.where(inside, ((pn * HI + eih) * WI + eiw) * C + lh * 16, -1)
                        got = np.where(in_zero, -1, src[np.clip(unit, 0, g["PP"] * 64 - 1)])
                        need(~valid | (got == want), f"s2i OW={OW} N={N}: wrong tap bytes (kh={kh} kw={kw})")
                # the fused downsample reads conv1's centre tap (kh = kw = 1) = input (2 oh, 2 ow)


def max_batch_int32():
    """Largest batch whose input tensor offsets stay int32 in every kernel above."""
    lim = []
    for W, C in ((28, 128), (14, 256), (7, 512)):
        lim.append(INT_MAX // (W * W * C))
    for OW, C in ((28, 64), (14, 128), (7, 256)):
        lim.append(INT_MAX // (4 * OW * OW * C))
    return min(lim)


def run(batches):
    for N in batches:
        for W in (28, 14, 7):
            check_conv3x3i(W, N)
        for OW in (28, 14, 7):
            check_s2i(OW, N)
    return max_batch_int32()


if __name__ == "__main__":
    Ns = [int(a) for a in sys.argv[1:]] or [1, 2, 3, 5, 8, 17, 256]
    mb = run(Ns)
    print(f"dma plans ok for N in {Ns}; int32 offsets hold up to N = {mb}")
