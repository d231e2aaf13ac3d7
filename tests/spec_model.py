"""Textbook 3GPP model of the PDSCH coding chain — TEST INFRASTRUCTURE ONLY.

Written from the specification's definitions (bit lists, polynomials, matrices), deliberately
unlike the oracle's implementation, to pin the oracle's coding stages where the reference's
own translation units cannot be built here ("Oracle and pinning"):

  crc24(bits, poly)       36.212 5.1.1  (CRC24A / CRC24B generator polynomials)
  turbo_encode(c, f1, f2) 36.212 5.1.3.2 (PCCC, 8-state RSC g0 = 1+D^2+D^3, g1 = 1+D+D^3,
                          QPP interleaver, trellis termination), returned in the reference's
                          d layout: (x_k, z_k, z'_k) per bit, then the 12 tail bits
  subblock(d_streams)     36.212 5.1.4.1.1 (32-column interleaver, bitrev column permutation,
                          the pi(k) rule for d^(2)) and the bit collection w
  rate_match(...)         36.212 5.1.4.1.2 (Ncb, E per block, k0, circular selection)
  gold(c_init, n)         36.211 7.2 (length-31 Gold sequence, Nc = 1600)
  crs(...)                36.211 6.10.1 (cell-specific reference signals: sequence and mapping)
  alamouti_grid(...)      36.211 6.3.4.3 / 6.3.5 (transmit diversity layer pairs on consecutive
                          data REs), with the reference's fixed-point scaling rules

Pure Python loops: use the small sizes of the CPU suite.
"""
import numpy as np

NULL = 2
CRC24A = [24, 23, 18, 17, 14, 11, 10, 7, 6, 5, 4, 3, 1, 0]
CRC24B = [24, 23, 6, 5, 1, 0]
COLPERM = [0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30,
           1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31]


def bytes_to_bits(data, nbits):
    """MSB-first bit list (a_0 is the MSB of byte 0)."""
    return [(data[i >> 3] >> (7 - (i & 7))) & 1 for i in range(nbits)]


def crc24(bits, taps):
    """Parity bits p_0..p_23 of 36.212 5.1.1: a(D) D^24 mod g(D), highest power first."""
    g = [0] * 25
    for t in taps:
        g[24 - t] = 1          # g[0] is the D^24 coefficient
    reg = list(bits) + [0] * 24
    for i in range(len(bits)):
        if reg[i]:
            for j in range(25):
                reg[i + j] ^= g[j]
    return reg[len(bits):]


def qpp(K, f1, f2):
    return [(f1 * i + f2 * i * i) % K for i in range(K)]


def _rsc(bits):
    """8-state RSC of 36.212 5.1.3.2.1: returns (z, tail_x, tail_z)."""
    s = [0, 0, 0]                       # shift register contents D^1, D^2, D^3
    z = []
    for c in bits:
        a = c ^ s[1] ^ s[2]             # feedback g0 = 1 + D^2 + D^3
        z.append(a ^ s[0] ^ s[2])       # output g1 = 1 + D + D^3
        s = [a, s[0], s[1]]
    tx, tz = [], []
    for _ in range(3):                  # termination: input = feedback, so a = 0
        x = s[1] ^ s[2]
        tx.append(x)
        tz.append(s[0] ^ s[2])
        s = [0, s[0], s[1]]
    return z, tx, tz


def turbo_encode(c_bits, f1, f2):
    """d in the reference layout (3K + 12 entries)."""
    K = len(c_bits)
    pi = qpp(K, f1, f2)
    z, tx, tz = _rsc(c_bits)
    z2, tx2, tz2 = _rsc([c_bits[pi[i]] for i in range(K)])
    d = []
    for k in range(K):
        d += [c_bits[k], z[k], z2[k]]
    for i in range(3):
        d += [tx[i], tz[i]]
    for i in range(3):
        d += [tx2[i], tz2[i]]
    return d


def streams_from_d(d, K):
    """d^(0), d^(1), d^(2) (length D = K + 4 each) from the interleaved d layout."""
    D = K + 4
    return [[d[3 * k + s] for k in range(D)] for s in range(3)]


def subblock(streams):
    """v^(0), v^(1), v^(2) and w (36.212 5.1.4.1.1 / 5.1.4.1.2)."""
    D = len(streams[0])
    R = (D + 31) // 32
    Kpi = 32 * R
    ND = Kpi - D
    ys = [[NULL] * ND + list(st) for st in streams]
    v = []
    for s in (0, 1):
        y = ys[s]
        v.append([y[32 * row + COLPERM[col]] for col in range(32) for row in range(R)])
    y2 = ys[2]
    v.append([y2[(COLPERM[k // R] + 32 * (k % R) + 1) % Kpi] for k in range(Kpi)])
    w = list(v[0])
    for k in range(Kpi):
        w += [v[1][k], v[2][k]]
    return R, w


def rate_match(w, R, G, C, r, Qm, Nl=1, rv=0, Nsoft=1827072, Kmimo=1, Mdlharq=8, limited=False):
    """e_0..e_{E-1} of code block r; None when Ncb < Kw (the reference's limited-buffer exit) unless
    `limited` (36.212's own limited-buffer rule, the build's opt-in extension)."""
    Kw = 3 * 32 * R
    Nir = Nsoft // (Kmimo * min(Mdlharq, 8))
    Ncb = min(Nir // C, Kw)
    if Ncb < Kw and not limited:
        return None
    Gp = G // (Nl * Qm)
    gamma = Gp % C
    E = Nl * Qm * (Gp // C) if r <= C - gamma - 1 else Nl * Qm * (-(-Gp // C))
    k0 = R * (2 * (-(-Ncb // (8 * R))) * rv + 2)
    e, j = [], 0
    while len(e) < E:
        x = w[(k0 + j) % Ncb]
        if x != NULL:
            e.append(x)
        j += 1
    return e


def gold(c_init, n):
    """c(0..n-1) of 36.211 7.2."""
    Nc = 1600
    x1 = [1] + [0] * 30
    x2 = [(c_init >> i) & 1 for i in range(31)]
    for m in range(Nc + n - 31):
        x1.append(x1[m + 3] ^ x1[m])
        x2.append(x2[m + 3] ^ x2[m + 2] ^ x2[m + 1] ^ x2[m])
    return [x1[i + Nc] ^ x2[i + Nc] for i in range(n)]


def crs(N_RB, Nid, subframe, port, amp, N, first_carrier, Ncp=0):
    """Cell-specific RS of one subframe, 36.211 6.10.1 (normal CP): {(l, fft_bin): (I, Q)} with the
    QPSK amplitude (amp * 23170) >> 15.  Subcarrier k maps to bin first_carrier + k below DC and
    to k - 6 N_RB + 1 above it (the DC bin is skipped)."""
    a = (amp * 23170) >> 15
    out = {}
    nsymb = 7
    for slot in (0, 1):
        ns = 2 * subframe + slot
        for lsym in (0, nsymb - 3):
            c_init = (1 << 10) * (7 * (ns + 1) + lsym + 1) * (2 * Nid + 1) + 2 * Nid + (1 - Ncp)
            c = gold(c_init, 4 * 110)
            if port == 0:
                nu = 0 if lsym == 0 else 3
            else:
                nu = 3 if lsym == 0 else 0
            for m in range(2 * N_RB):
                mp = m + 110 - N_RB
                k = 6 * m + (nu + Nid % 6) % 6
                fbin = first_carrier + k if k < 6 * N_RB else k - 6 * N_RB + 1
                out[(slot * nsymb + lsym, fbin)] = (a * (1 - 2 * c[2 * mp]), a * (1 - 2 * c[2 * mp + 1]))
    return out


# ------------------------------------------------------------------ transmit diversity (36.211 6.3.4.3)
def _w16(v):
    return ((int(v) + 32768) & 0xFFFF) - 32768


# QAM levels in Q15 (16-QAM: 1/sqrt10 (2 +- 1); 64-QAM: 1/sqrt42 (4 +- (2 +- 1))).  The reference
# keeps them in int tables (LTE_TRANSPORT/vars.h:72, filled by dlsch_modulation.c:79-103), so the
# outermost 64-QAM level 7/sqrt42 = 35393 stays > 32767 until it is scaled by amp >> 15.
QAM16_RAW = {}
QAM64_RAW = {}
for _a in (-1, 1):
    for _b in (-1, 1):
        QAM16_RAW[(1 + _a) + (1 + _b) // 2] = -_a * (20724 + _b * 10362)
        for _c in (-1, 1):
            QAM64_RAW[(1 + _a) * 2 + (1 + _b) + (1 + _c) // 2] = -_a * (20225 + _b * (10112 + _c * 5056))


def _sym_index(bits, Qm):
    """(re, im) level indices of one QAM symbol: bit pairs alternate re / im, MSB weight first."""
    ir = ii = 0
    for j in range(0, Qm, 2):
        w = 1 << ((Qm - 2 - j) >> 1)
        ir += w * bits[j]
        ii += w * bits[j + 1]
    return ir, ii


def alamouti_grid(e, N_RB, N, first_carrier, nushift, npdcch, Qm, amp=512, srho=8192):
    """Transmit-diversity RE grid of one subframe (2 antennas, even N_RB, no PBCH/sync
    exclusions): layer pairs x(2i), x(2i+1) go to consecutive data REs in frequency-first order
    (36.211 6.3.4.3, 6.3.5): RE 2i: (x0, -x1*)/sqrt2, RE 2i+1: (x1, x0*)/sqrt2, in the
    reference's fixed point (dlsch_modulation.c:362-546): amp_rho = amp*rho >> 13; QPSK +-g with
    g = amp_rho/sqrt2 then a second 1/sqrt2 after the sign; QAM (amp_rho/sqrt2) * level >> 15
    with the conjugate's negation applied after the scaling."""
    ampr = (amp * srho) >> 13
    g = (ampr * 23170) >> 15
    a2 = (ampr * 23170) >> 15
    raw = QAM16_RAW if Qm == 4 else QAM64_RAW
    grid = np.zeros((2, 14 * N, 2), dtype=np.int64)
    v = nushift % 3
    pos = 0
    for l in range(npdcch, 14):
        pil = l in (4, 7, 11)
        data = []
        for rb in range(N_RB):
            off = first_carrier + 12 * rb
            if off >= N:
                off = off - N + 1              # past DC (even N_RB)
            for re in range(12):
                if pil and re in (v, v + 3, v + 6, v + 9):
                    continue
                data.append(l * N + off + re)
        assert len(data) % 2 == 0
        for i in range(0, len(data), 2):
            xa = [int(b) for b in e[pos:pos + Qm]]
            xb = [int(b) for b in e[pos + Qm:pos + 2 * Qm]]
            pos += 2 * Qm
            if Qm == 2:
                ta = (((-g if xa[0] else g) * 23170) >> 15, ((-g if xa[1] else g) * 23170) >> 15)
                tb = (((g if xb[0] else -g) * 23170) >> 15, ((-g if xb[1] else g) * 23170) >> 15)
            else:
                ra, ia = _sym_index(xa, Qm)
                rb_, ib = _sym_index(xb, Qm)
                ta = ((a2 * raw[ra]) >> 15, (a2 * raw[ia]) >> 15)
                tb = (-((a2 * raw[rb_]) >> 15), (a2 * raw[ib]) >> 15)
            n, m = data[i], data[i + 1]
            grid[0, n] = ta
            grid[1, n] = tb
            grid[0, m] = (_w16(-tb[0]), tb[1])
            grid[1, m] = (ta[0], _w16(-ta[1]))
    out = (grid[..., 0] & 0xFFFF) | ((grid[..., 1] & 0xFFFF) << 16)
    return out.astype(np.uint32).view(np.int32), pos


# ------------------------------------------------------------------ 4-port large-delay CDD (36.211 6.3.4.2.2)
# Codebook for 4 antenna ports, Table 6.3.4.2.3-2: W_n = I - 2 u_n u_n^H / (u_n^H u_n); the rank-2
# entry of n = 12, 13, 14, 15 takes the columns {1,2}, {1,3}, {1,3}, {1,2} (scaled by 1/sqrt2).
U_N = {12: (1, -1, -1, 1), 13: (1, -1, 1, -1), 14: (1, 1, -1, -1), 15: (1, 1, 1, 1)}
RANK2_COLS = {12: (0, 1), 13: (0, 2), 14: (0, 2), 15: (0, 1)}


def householder(n):
    from fractions import Fraction
    u = U_N[n]
    nn = sum(x * x for x in u)
    return [[Fraction(int(i == j)) - Fraction(2 * u[i] * u[j], nn) for j in range(4)] for i in range(4)]


def cdd4_precode(i, x0, x1):
    """y_p (p = 0..3) of layer-symbol i for complex layers x0, x1 (integer pairs): y = W(i) D(i) U x(i)
    with U = [[1,1],[1,-1]]/sqrt2, D(i) = diag(1, e^{-j pi i}), W(i) = C_k/sqrt2, C_k the rank-2
    codebook matrix of index 12 + (floor(i/2) mod 4); the two 1/sqrt2 combine to 1/2.  Exact
    rational arithmetic, rounded down per component."""
    import math
    n = 12 + (i // 2) % 4
    Wn = householder(n)
    c0, c1 = RANK2_COLS[n]
    s = -1 if i % 2 else 1
    v = [(x0[0] + x1[0], x0[1] + x1[1]), (s * (x0[0] - x1[0]), s * (x0[1] - x1[1]))]   # D U x, times sqrt2
    out = []
    for p in range(4):
        re = (Wn[p][c0] * v[0][0] + Wn[p][c1] * v[1][0]) / 2
        im = (Wn[p][c0] * v[0][1] + Wn[p][c1] * v[1][1]) / 2
        out.append((_w16(math.floor(re)), _w16(math.floor(im))))
    return out


def cdd4_grid(e0, e1, N_RB, N, first_carrier, nushift, npdcch, Qm, amp=512, srho=8192):
    """4-antenna large-delay CDD RE grid of one subframe (2 codewords of one layer each, even
    N_RB, no PBCH/sync exclusions).  Data REs in frequency-first order skip the CRS of ports 0/1
    (symbols 0, 4, 7, 11) and 2/3 (symbols 1, 8): nu_shift mod 3 + {0, 3, 6, 9} in each RB.
    QAM levels as the reference's LARGE_CDD branch: (raw level * amp_rho) >> 15."""
    ampr = (amp * srho) >> 13
    raw = QAM16_RAW if Qm == 4 else QAM64_RAW
    grid = np.zeros((4, 14 * N, 2), dtype=np.int64)
    v = nushift % 3
    pos = i = 0
    for l in range(npdcch, 14):
        pil = l in (1, 4, 7, 8, 11)
        for rb in range(N_RB):
            off = first_carrier + 12 * rb
            if off >= N:
                off = off - N + 1
            for re in range(12):
                if pil and re in (v, v + 3, v + 6, v + 9):
                    continue
                xs = []
                for e in (e0, e1):
                    b = [int(x) for x in e[pos:pos + Qm]]
                    if Qm == 2:
                        g = (ampr * 23170) >> 15
                        xs.append((-g if b[0] else g, -g if b[1] else g))
                    else:
                        ir, ii = _sym_index(b, Qm)
                        xs.append(((raw[ir] * ampr) >> 15, (raw[ii] * ampr) >> 15))
                pos += Qm
                for p, y in enumerate(cdd4_precode(i, xs[0], xs[1])):
                    grid[p, l * N + off + re] = y
                i += 1
    out = (grid[..., 0] & 0xFFFF) | ((grid[..., 1] & 0xFFFF) << 16)
    return out.astype(np.uint32).view(np.int32), i


def crs_p23(N_RB, Nid, subframe, port, amp, N, first_carrier, Ncp=0):
    """CRS of antenna port 2 or 3 (36.211 6.10.1.2): symbol l = 1 of each slot, nu = 3 (ns mod 2)
    (port 2) or 3 + 3 (ns mod 2) (port 3); same sequence rule as crs() with l = 1."""
    a = (amp * 23170) >> 15
    out = {}
    nsymb = 7 if Ncp == 0 else 6
    for slot in (0, 1):
        ns = 2 * subframe + slot
        c_init = (1 << 10) * (7 * (ns + 1) + 1 + 1) * (2 * Nid + 1) + 2 * Nid + (1 - Ncp)
        c = gold(c_init, 4 * 110)
        nu = (0 if port == 2 else 3) + 3 * (ns % 2)
        for m in range(2 * N_RB):
            mp = m + 110 - N_RB
            k = 6 * m + (nu + Nid % 6) % 6
            fbin = first_carrier + k if k < 6 * N_RB else k - 6 * N_RB + 1
            out[(slot * nsymb + 1, fbin)] = (a * (1 - 2 * c[2 * mp]), a * (1 - 2 * c[2 * mp + 1]))
    return out


def pcfich(N_RB, Nid, subframe, cfi, amp, N, first_carrier, mode1, n_ant):
    """PCFICH REs of symbol 0 per antenna: {grid index: (re, im)} (36.212 5.3.4 CFI codeword,
    36.211 6.7.1 scrambling, 7.1.2 QPSK, 6.3.3.3 / 6.3.4.3 transmit diversity, 6.7.4 mapping to
    four REGs, 6.2.4 REGs of symbol 0 skipping the port-0/1 RS positions)."""
    cw = {1: (0, 1, 1), 2: (1, 0, 1), 3: (1, 1, 0)}[cfi]
    c = gold(((subframe + 1) * (2 * Nid + 1) << 9) + Nid, 32)
    bt = [cw[i % 3] ^ c[i] for i in range(32)]
    g = (amp * 23170) >> 15 if mode1 else int(amp / 2)
    x = [(-g if bt[2 * i] else g, -g if bt[2 * i + 1] else g) for i in range(16)]
    if mode1:
        y = [x, x]
    else:
        y0, y1 = [None] * 16, [None] * 16
        for k in range(0, 16, 2):
            a, b = x[k], x[k + 1]
            y0[k], y1[k] = a, (-b[0], b[1])            # x0, -x1*
            y0[k + 1], y1[k + 1] = b, (a[0], -a[1])    # x1,  x0*
        y = [y0, y1]
    kbar = 6 * (Nid % (2 * N_RB))
    vs = (Nid % 6) % 3
    out = [dict() for _ in range(n_ant)]
    m = 0
    for i in range(4):
        k0 = (kbar + (i * N_RB // 2) * 6) % (12 * N_RB)
        for j in range(6):
            if j in (vs, vs + 3):
                continue
            idx = first_carrier + k0 + j
            if idx >= N:
                idx = idx - N + 1                      # DC skip
            for a in range(n_ant):
                out[a][idx] = y[a][m]
            m += 1
    return out


# ------------------------------------------------------------------ whole DLSCH chain (36.212 5.3.2)
def _qpp_params():
    import os
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                            "oai4g_qpp.c")).read()
    return {int(a): (int(b), int(c)) for a, b, c in re.findall(r"\{\s*(\d+)\s*,\s*(\d+)\s*,\s*(\d+)\s*\}", src)}


def segment(b):
    """36.212 5.1.2 code block segmentation of the bit list b (TB + CRC24A): returns the code
    blocks (lists of K_r bits, CRC24B appended when C > 1) and F.  Filler bits are zeros: the
    reference encodes them as 0 rather than <NULL> (A6q, 3gpplte_sse.c:380-476; the oracle and
    the reference TU agree, tests/test_ref_pin_cpu.py)."""
    Ks = sorted(_qpp_params())
    Z = 6144
    B = len(b)
    if B <= Z:
        C, Bp = 1, B
    else:
        C = -(-B // (Z - 24))
        Bp = B + 24 * C
    Kp = min(K for K in Ks if C * K >= Bp)
    if C == 1:
        Cp, Km, Cm = 1, 0, 0
    else:
        Km = max(K for K in Ks if K < Kp)
        Cm = (C * Kp - Bp) // (Kp - Km)
        Cp = C - Cm
    F = Cp * Kp + Cm * Km - Bp
    blocks, s = [], 0
    for r in range(C):
        K = Km if r < Cm else Kp
        blk = [0] * (F if r == 0 else 0)
        n = K - len(blk) - (24 if C > 1 else 0)
        blk += list(b[s:s + n])
        s += n
        if C > 1:
            blk += crc24(blk, CRC24B)
        blocks.append(blk)
    return blocks, F


def dlsch_e(payload, TBS, G, Qm, Nl=1, rv=0, Kmimo=1, Mdlharq=8, c_init=None, Nsoft=1827072):
    """Scrambled bits e_0..e_{G-1} of one transport block: CRC24A, segmentation, turbo coding,
    sub-block interleaving, rate matching (E per block, concatenated) and the 36.211 6.3.1
    scrambling with the Gold sequence of c_init (None: unscrambled)."""
    f = _qpp_params()
    a = bytes_to_bits(payload, TBS)
    blocks, _ = segment(a + crc24(a, CRC24A))
    e = []
    for r, c in enumerate(blocks):
        K = len(c)
        R, w = subblock(streams_from_d(turbo_encode(c, *f[K]), K))
        er = rate_match(w, R, G, len(blocks), r, Qm, Nl=Nl, rv=rv, Kmimo=Kmimo, Mdlharq=Mdlharq, Nsoft=Nsoft)
        assert er is not None, "limited-buffer rate matching (Ncb < Kw): no reference output"
        e += er
    assert len(e) == G
    if c_init is not None:
        g = gold(c_init, G)
        e = [x ^ y for x, y in zip(e, g)]
    return e


# ------------------------------------------------------------------ PDSCH resource mapping (36.211 6.3.5)
def pdsch_res(N_RB, N, first_carrier, nushift, npdcch, subframe, crs_ports, Ncp=0, rb_alloc=None):
    """Data REs of one FDD subframe in the order 36.211 6.3.5 maps them: for each OFDM symbol
    l >= npdcch, increasing subcarrier k over the allocated PRBs.  Excluded: the CRS of the ports
    in use (6.10.1.2: k = 6m + (v + v_shift) mod 6 with v = 0 / 3 in symbols 0 / N_symb-3 of each
    slot, ports 0 and 1 swapped; 1 port when crs_ports == 1), PBCH (6.6.4: subframe 0, slot 1
    symbols 0-3, the 72 centre subcarriers) and the FDD synchronisation signals (6.11: subframes
    0 and 5, the last two symbols of slot 0, the 72 centre subcarriers).  Subcarrier k sits in FFT
    bin first_carrier + k below DC and k - 6 N_RB + 1 above it (the DC bin is unused).
    Returns a list of (l, bin, rb)."""
    nsymb = 14 if Ncp == 0 else 12
    nsl = nsymb // 2
    out = []
    for l in range(npdcch, nsymb):
        ls = l % nsl
        crs_sym = ls == 0 or ls == nsl - 3
        pbch = subframe == 0 and nsl <= l < nsl + 4
        sync = subframe in (0, 5) and l in (nsl - 2, nsl - 1)
        for rb in range(N_RB):
            if rb_alloc is not None and not (rb_alloc[rb >> 5] >> (rb & 31)) & 1:
                continue
            for kk in range(12):
                k = 12 * rb + kk
                if crs_sym:
                    if crs_ports == 1:
                        if k % 6 == ((0 if ls == 0 else 3) + nushift) % 6:
                            continue
                    elif k % 3 == nushift % 3:          # ports 0 and 1: v and v + 3
                        continue
                if (pbch or sync) and 6 * N_RB - 36 <= k < 6 * N_RB + 36:
                    continue
                b = first_carrier + k
                out.append((l, b if b < N else b - N + 1, rb))
    return out


def crs_symbol(l, Ncp=0):
    nsl = 7 if Ncp == 0 else 6
    return l % nsl in (0, nsl - 3)


def qam(bits, Qm, ampr, raw16=None, raw64=None):
    """One modulation symbol (36.211 7.1) in the reference's fixed point: QPSK +-(ampr/sqrt2)
    ((ampr * 23170) >> 15, bit 1 -> negative); 16/64-QAM (level * ampr) >> 15 with the levels
    kept as the reference's int Q15 tables (the 64-QAM 7/sqrt42 entry 35393 > 32767, see QAM64_RAW)."""
    if Qm == 2:
        g = (ampr * 23170) >> 15
        return (-g if bits[0] else g, -g if bits[1] else g)
    raw = QAM16_RAW if Qm == 4 else QAM64_RAW
    ir, ii = _sym_index(bits, Qm)
    return ((raw[ir] * ampr) >> 15, (raw[ii] * ampr) >> 15)


def _pack(grid):
    out = (grid[..., 0] & 0xFFFF) | ((grid[..., 1] & 0xFFFF) << 16)
    return out.astype(np.uint32).view(np.int32)


def siso_grid(e, res, Qm, n_ant, N, amp=512, srho_a=8192, srho_b=8192, Ncp=0):
    """Single-layer PDSCH grid of one subframe (36.211 6.3.4.1: one antenna port, no precoding):
    consecutive Qm bits -> one symbol -> the next RE of res.  PDSCH EPRE: rho_A in symbols without
    CRS, rho_B in symbols with CRS (36.213 5.2), amp_rho = (amp * sqrt_rho) >> 13 in Q13.  The
    reference writes the port-0 symbol to every TX antenna (dlsch_modulation.c:266-273)."""
    nsymb = 14 if Ncp == 0 else 12
    grid = np.zeros((n_ant, nsymb * N, 2), dtype=np.int64)
    ra, rb_ = (amp * srho_a) >> 13, (amp * srho_b) >> 13
    for i, (l, b, _) in enumerate(res):
        x = qam([int(v) for v in e[Qm * i:Qm * i + Qm]], Qm, rb_ if crs_symbol(l, Ncp) else ra)
        for a in range(n_ant):
            grid[a, l * N + b] = (_w16(x[0]), _w16(x[1]))
    return _pack(grid), Qm * len(res)


def cdd2_grid(e0, e1, res, Qm0, Qm1, N, amp=512, srho_a=8192, srho_b=8192, Ncp=0, sign_reset_per_rb=False):
    """Two-layer large-delay CDD on 2 antenna ports (36.211 6.3.4.2.2, codebook index 0):
    y(i) = W D(i) U x(i) with W = I/sqrt2, U = [[1, 1], [1, -1]]/sqrt2, D(i) = diag(1, (-1)^i),
    i.e. y0 = (x0 + x1)/2, y1 = (-1)^i (x0 - x1)/2; layer i of codeword q carries its codeword's
    i-th symbol (6.3.3.2, two codewords, one layer each).  Fixed-point rule of the reference
    (dlsch_modulation.c:720-727): floor halving of the int16 sums, sign applied after the
    floor, accumulated into int16.  The reference counts i per resource block (its sign s is
    reset to +1 at every allocate_REs_in_RB call, :198, :748): sign_reset_per_rb=True models that;
    the two agree whenever every RB contributes an even number of REs."""
    nsymb = 14 if Ncp == 0 else 12
    grid = np.zeros((2, nsymb * N, 2), dtype=np.int64)
    ra, rb_ = (amp * srho_a) >> 13, (amp * srho_b) >> 13
    prev, i_rb = None, 0
    for i, (l, b, rb) in enumerate(res):
        if (l, rb) != prev:
            prev, i_rb = (l, rb), 0
        ampr = rb_ if crs_symbol(l, Ncp) else ra
        x0 = qam([int(v) for v in e0[Qm0 * i:Qm0 * i + Qm0]], Qm0, ampr)
        x1 = qam([int(v) for v in e1[Qm1 * i:Qm1 * i + Qm1]], Qm1, ampr)
        s = -1 if (i_rb if sign_reset_per_rb else i) % 2 else 1
        grid[0, l * N + b] = (_w16((x0[0] + x1[0]) >> 1), _w16((x0[1] + x1[1]) >> 1))
        grid[1, l * N + b] = (_w16(s * ((x0[0] - x1[0]) >> 1)), _w16(s * ((x0[1] - x1[1]) >> 1)))
        i_rb += 1
    return _pack(grid), len(res)


# ------------------------------------------------------------------ PDCCH (36.212 5.3.3, 36.211 6.8)
CC_COLPERM = [1, 17, 9, 25, 5, 21, 13, 29, 3, 19, 11, 27, 7, 23, 15, 31,
              0, 16, 8, 24, 4, 20, 12, 28, 2, 18, 10, 26, 6, 22, 14, 30]   # 36.212 Table 5.1.4-2


def crc16_ref(bits):
    """CRC16 parity bits p_0..p_15 of 36.212 5.1.1 (g = D^16 + D^12 + D^5 + 1) for whole bytes.
    Departure (cited parameter): for a partial last byte the reference's crc16 (crc_byte.c:167-168)
    shifts the register by `resbit` and looks up a table entry indexed by the resbit-bit
    remainder, which is not the spec's polynomial division; the model reproduces that step."""
    g = [16, 12, 5, 0]
    n = len(bits)
    full = n - n % 8
    reg = 0                                          # 16-bit register, MSB = oldest
    for b in bits[:full]:
        fb = ((reg >> 15) & 1) ^ b
        reg = (reg << 1) & 0xFFFF
        if fb:
            reg ^= 0x1021
    r = n % 8
    if r:
        tab = _crc16_byte_table()
        v = 0
        for b in bits[full:]:
            v = (v << 1) | b
        crc32 = reg << 16
        crc32 = ((crc32 << r) & 0xFFFFFFFF) ^ (tab[(v ^ (crc32 >> (32 - r))) & 0xFF] << 16)
        reg = (crc32 >> 16) & 0xFFFF
    return [(reg >> (15 - i)) & 1 for i in range(16)]


_C16 = []


def _crc16_byte_table():
    if not _C16:
        for v in range(256):
            reg = 0
            for i in range(8):
                fb = ((reg >> 15) & 1) ^ ((v >> (7 - i)) & 1)
                reg = (reg << 1) & 0xFFFF
                if fb:
                    reg ^= 0x1021
            _C16.append(reg)
    return _C16


def tbcc_encode(c):
    """36.212 5.1.3.1 tail-biting convolutional code, g0 = 133, g1 = 171, g2 = 165 (octal): the
    register starts with the last six input bits; returns d in the reference layout
    (d^(0)_k, d^(1)_k, d^(2)_k per k)."""
    G = [[(g >> (6 - j)) & 1 for j in range(7)] for g in (0o133, 0o171, 0o165)]
    K = len(c)
    d = []
    for k in range(K):
        taps = [c[(k - j) % K] for j in range(7)]     # c_k, c_{k-1}, ... (tail-biting wrap)
        for i in range(3):
            d.append(sum(G[i][j] & taps[j] for j in range(7)) & 1)
    return d


def cc_rate_match(d, E):
    """36.212 5.1.4.2: sub-block interleaving of each stream (Table 5.1.4-2 permutation, <NULL>
    padding in front), w = v0 || v1 || v2, circular selection skipping <NULL>."""
    D = len(d) // 3
    R = -(-D // 32)
    ND = 32 * R - D
    w = []
    for s in range(3):
        y = [NULL] * ND + d[s::3]
        w += [y[32 * row + CC_COLPERM[col]] for col in range(32) for row in range(R)]
    e, k = [], 0
    while len(e) < E:
        if w[k % len(w)] != NULL:
            e.append(w[k % len(w)])
        k += 1
    return e


def dci_bits(pdu, length):
    """The DCI payload a_0..a_{A-1}: generate_dci0 reads the DCI_ALLOC_t pdu bytes in reverse
    order (dci.c:233-251, the little-endian bit-field struct) and takes the first A bits MSB-first."""
    flip = list(reversed(list(pdu[:4]))) if length <= 32 else list(reversed(list(pdu[:8])))
    return bytes_to_bits(flip, length)


def dci_e(pdu, length, L, rnti):
    """36.212 5.3.3: CRC16 attachment with the RNTI mask, TBCC, rate matching to 72 * 2^L bits."""
    a = dci_bits(pdu, length)
    p = crc16_ref(a)
    x = [(rnti >> (15 - i)) & 1 for i in range(16)]
    c = a + [p[i] ^ x[i] for i in range(16)]
    return cc_rate_match(tbcc_encode(c), 72 << L)


def n_reg_pdcch(N_RB, npdcch, n_ant=2):
    """REGs of the control region (36.211 6.2.4): 2 per RB in symbol 0 (and symbol 1 with 4 ports),
    3 per RB elsewhere (normal CP)."""
    return sum((2 if (l == 0 or (l == 1 and n_ant == 4)) else 3) * N_RB for l in range(npdcch))


def phich_regs(N_RB, Nid, Ng6, pcfich_regs):
    """36.211 6.9.3, normal duration, normal CP: PHICH group m' uses REG n_bar_i of symbol 0,
    n_bar_i = (Nid + m' + floor(i n_0 / 3)) mod n_0 counted over the REGs of symbol 0 NOT used by
    PCFICH; returned as absolute REG indices of symbol 0 (units of 6 subcarriers)."""
    ngroup = -(-Ng6 * N_RB // 48)
    free = [r for r in range(2 * N_RB) if r not in pcfich_regs]
    n0 = len(free)
    return [[free[(Nid + m + (i * n0) // 3) % n0] for i in range(3)] for m in range(ngroup)]


def pdcch_grid(N_RB, Nid, subframe, dcis, npdcch, amp, N, first_carrier, mode1, n_ant, Ng6=6):
    """PDCCH REs of the control region per antenna {grid index within the subframe: (re, im)}
    (36.211 6.8.2 multiplexing with <NIL>, 6.8.2 scrambling c_init = ns/2 2^9 + Nid, 7.1.2 QPSK,
    6.3.3.3 / 6.3.4.3 transmit diversity, 6.8.5 quadruplet interleaving (36.212 5.1.4.2.1 with the
    <NULL>s removed) and cyclic shift by Nid, REG mapping frequency-first over k' then l' skipping
    the PCFICH and PHICH REGs; normal CP, normal PHICH duration).  dcis: (pdu, length, L, nCCE,
    rnti).  Departures (cited parameters): <NIL> quadruplets carry 0 with one port and +g on both
    bits with two (dci.c:2182-2224), gains as PCFICH (amp 23170 >> 15, amp / 2)."""
    nreg = n_reg_pdcch(N_RB, npdcch, n_ant)
    kbar = 6 * (Nid % (2 * N_RB))
    pcf = [((kbar + (i * N_RB // 2) * 6) % (12 * N_RB)) // 6 for i in range(4)]
    ph = phich_regs(N_RB, Nid, Ng6, pcf)
    ph_set = {r for g in ph for r in g}
    nquad = nreg - 4 - 3 * len(ph)
    Mbits = 8 * nquad
    b = [NIL] * Mbits
    for pdu, length, L, ncce, rnti in dcis:
        if ncce < 0:                                 # no free candidate in the search space: not sent
            continue
        e = dci_e(pdu, length, L, rnti)
        b[72 * ncce:72 * ncce + len(e)] = e
    b = b[:Mbits]
    c = gold((subframe << 9) + Nid, Mbits)
    b = [x if x == NIL else x ^ c[i] for i, x in enumerate(b)]
    g = (amp * 23170) >> 15 if mode1 else int(amp / 2)
    nsym = Mbits // 2
    if mode1:
        d = [(0 if b[2 * i] == NIL else (-g if b[2 * i] else g), 0 if b[2 * i + 1] == NIL else (-g if b[2 * i + 1] else g))
             for i in range(nsym)]
        y = [d, d]
    else:
        s = [(-g if x == 1 else g) for x in b]     # <NIL> -> +g
        y0, y1 = [None] * nsym, [None] * nsym
        for i in range(0, nsym, 2):
            x0, x1 = (s[2 * i], s[2 * i + 1]), (s[2 * i + 2], s[2 * i + 3])
            y0[i], y1[i] = x0, (-x1[0], x1[1])
            y0[i + 1], y1[i + 1] = x1, (x0[0], -x0[1])
        y = [y0, y1]
    # quadruplet interleaving (36.212 5.1.4.2.1 on quadruplets, <NULL> removed) + cyclic shift
    R = -(-nquad // 32)
    ND = 32 * R - nquad
    seq = [None] * ND + list(range(nquad))
    perm = [seq[32 * row + CC_COLPERM[col]] for col in range(32) for row in range(R)]
    perm = [p for p in perm if p is not None]
    wbar = [perm[(i + Nid) % nquad] for i in range(nquad)]
    out = [dict() for _ in range(n_ant)]
    vs = (Nid % 6) % 3
    m = 0
    for kp in range(12 * N_RB):
        for lp in range(npdcch):
            if lp == 0:                                  # REGs of 6 REs around the port-0/1 RS
                if kp % 6 or kp // 6 in pcf or kp // 6 in ph_set:
                    continue
                res = [kp + j for j in range(6) if j not in (vs, vs + 3)]
            else:
                if kp % 4:
                    continue
                res = [kp + j for j in range(4)]
            q = wbar[m]
            for j, k in enumerate(res):
                idx = first_carrier + k
                if idx >= N:
                    idx = idx - N + 1
                for a in range(n_ant):
                    out[a][lp * N + idx] = y[min(a, 1)][4 * q + j]
            m += 1
    assert m == nquad
    return out


NIL = 3


# ------------------------------------------------------------------ synchronisation signals (36.211 6.11)
def _bin(k, N_RB, N, first_carrier):
    """FFT bin of subcarrier k (0 .. 12 N_RB - 1): below DC from first_carrier, above it from 1."""
    return first_carrier + k if k < 6 * N_RB else k - 6 * N_RB + 1


def pss_seq(Nid2):
    """36.211 6.11.1.1 Zadoff-Chu d_u(n), u = 25 / 29 / 34, as (re, im) in Q15 with the reference
    table's rounding floor(32767 x) (cited parameter: PHY/LTE_REFSIG/primary_synch.h)."""
    import math
    u = (25, 29, 34)[Nid2]
    out = []
    for n in range(62):
        m = n if n < 31 else n + 1
        ang = -math.pi * u * m * (m + 1) / 63
        out.append((math.floor(32767 * math.cos(ang)), math.floor(32767 * math.sin(ang))))
    return out


def sss_seq(Nid, subframe5):
    """36.211 6.11.2.1: d(2n) / d(2n+1) from the m-sequences s, c, z (values +-1)."""
    def mseq(taps):
        x = [0, 0, 0, 0, 1]
        for i in range(26):
            x.append(sum(x[i + t] for t in taps) % 2)
        return [1 - 2 * v for v in x]
    st, ct, zt = mseq((2, 0)), mseq((3, 0)), mseq((4, 2, 1, 0))
    n1, n2 = Nid // 3, Nid % 3
    qp = n1 // 30
    q = (n1 + qp * (qp + 1) // 2) // 30
    mp = n1 + q * (q + 1) // 2
    m0 = mp % 31
    m1 = (m0 + mp // 31 + 1) % 31
    d = [0] * 62
    for n in range(31):
        s0, s1 = st[(n + m0) % 31], st[(n + m1) % 31]
        c0, c1 = ct[(n + n2) % 31], ct[(n + n2 + 3) % 31]
        z0, z1 = zt[(n + m0 % 8) % 31], zt[(n + m1 % 8) % 31]
        if not subframe5:
            d[2 * n], d[2 * n + 1] = s0 * c0, s1 * c1 * z0
        else:
            d[2 * n], d[2 * n + 1] = s1 * c0, s0 * c1 * z1
    return d


def sync_grid(N_RB, Nid, amp, N, first_carrier, n_ant, Ncp=0):
    """PSS and SSS of subframes 0 and 5 (FDD, 36.211 6.11.1.2 / 6.11.2.2): {(subframe, l, bin):
    (re, im)}, the same on every antenna; a = amp (one antenna) or (amp 23170) >> 15, PSS values
    (a d) >> 15 in Q15, SSS values a d (+-a, imaginary 0)."""
    a = amp if n_ant == 1 else (amp * 23170) >> 15
    nsl = 7 if Ncp == 0 else 6
    ps = pss_seq(Nid % 3)
    out = {}
    for sf in (0, 5):
        ss = sss_seq(Nid, sf == 5)
        for n in range(62):
            b = _bin(n - 31 + 6 * N_RB, N_RB, N, first_carrier)
            out[(sf, nsl - 1, b)] = ((a * ps[n][0]) >> 15, (a * ps[n][1]) >> 15)
            out[(sf, nsl - 2, b)] = (_w16(a * ss[n]), 0)
    return out


# ------------------------------------------------------------------ PBCH (36.212 5.3.1, 36.211 6.6)
def pbch_e(pdu, Nid, n_ant_enb, mode1, Ncp=0):
    """The scrambled PBCH bits of one 40 ms period: a = the 24 MIB bits (the reference's pdu bytes
    in reverse order, pbch.c:214-215), CRC16 XOR the antenna mask (36.212 Table 5.3.1.1-1: 0,
    all-ones, 0101...; the reference applies none in transmission mode 1), TBCC, rate matching to
    1920 (1728) bits, scrambling with c_init = Nid (36.211 6.6.1)."""
    a = bytes_to_bits(list(reversed(list(pdu[:3]))), 24)
    mask = 0 if mode1 else {1: 0, 2: 0xFFFF, 4: 0x5555}[n_ant_enb]
    p = crc16_ref(a)
    c = a + [p[i] ^ ((mask >> (15 - i)) & 1) for i in range(16)]
    E = 1920 if Ncp == 0 else 1728
    e = cc_rate_match(tbcc_encode(c), E)
    cs = gold(Nid, E)
    return [e[i] ^ cs[i] for i in range(E)]


def pbch_grid(pdu, frame_mod4, N_RB, Nid, amp, N, first_carrier, mode1, n_ant, n_ant_enb=2, Ncp=0):
    """PBCH REs of subframe 0 per antenna, {(l, bin): (re, im)}: quarter frame_mod4 of pbch_e,
    QPSK (7.1.2) with gain g = (amp 23170) >> 15, the 72 subcarriers around DC of symbols 0..3 of
    slot 1 minus the positions reserved for the RS of ports 0..3 (k = v_shift mod 3 + 3j in the
    symbols that carry them), k first then l (6.6.4).  Two antennas: SFBC (6.3.4.3) with the
    reference's fixed point (cited departures, pbch.c:116-145): each component (+-g 23170) >> 15
    (floor, so -g maps to one LSB more than +g), and the partner RE written as the negated /
    conjugated values of RE n."""
    E = 1920 if Ncp == 0 else 1728
    e = pbch_e(pdu, Nid, n_ant_enb, mode1, Ncp)[frame_mod4 * (E // 4):(frame_mod4 + 1) * (E // 4)]
    g = (amp * 23170) >> 15
    nsl = 7 if Ncp == 0 else 6
    pil_l = {0, 1} | ({3} if Ncp else set())        # slot-1 symbols carrying RS of ports 0..3
    vs3 = (Nid % 6) % 3
    res = []
    for lp in range(4):
        for kp in range(72):
            if lp in pil_l and kp % 3 == vs3:
                continue
            res.append((nsl + lp, _bin(6 * N_RB - 36 + kp, N_RB, N, first_carrier)))
    qp = [(-g if e[2 * i] else g, -g if e[2 * i + 1] else g) for i in range(len(res))]
    out = [dict() for _ in range(n_ant)]
    if mode1:
        for i, r in enumerate(res):
            for aa in range(n_ant):
                out[aa][r] = qp[i]
        return out
    s = lambda v: (v * 23170) >> 15
    for i in range(0, len(res), 2):
        x0, x1 = qp[i], qp[i + 1]
        y0 = (s(x0[0]), s(x0[1]))
        y1 = (s(-x1[0]), s(x1[1]))                   # -x1*
        out[0][res[i]], out[1][res[i]] = y0, y1
        out[0][res[i + 1]] = (_w16(-y1[0]), y1[1])    # x1
        out[1][res[i + 1]] = (y0[0], _w16(-y0[1]))    # x0*
    return out


# ------------------------------------------------------------------ PHICH (36.212 5.3.5, 36.211 6.9)
PHICH_W = [(1, 1, 1, 1), (1, -1, 1, -1), (1, 1, -1, -1), (1, -1, -1, 1),
           ('j', 'j', 'j', 'j'), ('j', '-j', 'j', '-j'), ('j', 'j', '-j', '-j'), ('j', '-j', '-j', 'j')]


def phich_grid(N_RB, Nid, subframe, ngroup, nseq, hi, amp, N, first_carrier, mode1, n_ant, pcfich_regs, Ng6=1,
               ref_c_init=True):
    """One PHICH of symbol 0 (normal CP, normal duration) per antenna, {bin: (re, im)} accumulated:
    HI repeated 3 times (5.3.5), BPSK z = (1 + j)(1 - 2b) in units of the gain, orthogonal
    sequence w (Table 6.9.1-2) and scrambling (1 - 2c(i)) per symbol (6.9.1), SISO gain
    (amp 23170) >> 15 or SFBC with amp / 2 (6.3.4.3), quadruplet i on REG n_bar_i (6.9.3).
    ref_c_init: the reference's c_init = ((subframe + 1)(Nid + 1)) 2^9 + Nid (phich.c:440) instead
    of the spec's (subframe + 1)(2 Nid + 1) 2^9 + Nid (cited departure)."""
    ci = (((subframe + 1) * (Nid + 1)) << 9) + Nid if ref_c_init else (((subframe + 1) * (2 * Nid + 1)) << 9) + Nid
    c = gold(ci, 12)
    b = 1 if hi else 0
    d = []
    for i in range(12):
        v = (1 - 2 * c[i]) * (1 - 2 * b)
        w = PHICH_W[nseq][i % 4]
        if w in (1, -1):
            d.append((w * v, w * v))
        else:
            sgn = 1 if w == 'j' else -1
            d.append((-sgn * v, sgn * v))                  # j (1 + j) = -1 + j
    g = (amp * 23170) >> 15 if mode1 else amp // 2
    if mode1:
        y = [[(_w16(x[0] * g), _w16(x[1] * g)) for x in d]] * n_ant
    else:
        y0, y1 = [None] * 12, [None] * 12
        for k in range(0, 12, 2):
            a0 = (_w16(d[k][0] * g), _w16(d[k][1] * g))
            b1 = (_w16(-d[k + 1][0] * g), _w16(d[k + 1][1] * g))
            y0[k], y1[k] = a0, b1
            y0[k + 1], y1[k + 1] = (_w16(-b1[0]), b1[1]), (a0[0], _w16(-a0[1]))
        y = [y0, y1]
    regs = phich_regs(N_RB, Nid, Ng6, pcfich_regs)[ngroup]
    vs = (Nid % 6) % 3
    out = [dict() for _ in range(n_ant)]
    for q in range(3):
        ro = first_carrier + 6 * regs[q]
        if ro > N:
            ro -= N - 1                                     # '>' (phich.c:560), not '>='
        m = 0
        for j in range(6):
            if j in (vs, vs + 3):
                continue
            for a in range(n_ant):
                r0, i0 = out[a].get(ro + j, (0, 0))
                out[a][ro + j] = (_w16(r0 + y[a][4 * q + m][0]), _w16(i0 + y[a][4 * q + m][1]))
            m += 1
    return out
