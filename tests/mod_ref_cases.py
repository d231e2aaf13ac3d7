"""Cases of the dlsch_modulation / dlsch_scrambling reference fixtures (tests/golden/mod_ref.json,
made by tests/golden/gen_mod_ref.py with the reference's own dlsch_modulation.c and
dlsch_scrambling.c compiled here, oracle/_ref/libref_mod.so).  Inputs are generated, not stored: e
bits from splitmix64 (rm_ref_cases), so the GPU box rebuilds them from the case list alone.

PCFICH cases (pcfich.c, the same library): a frame, CFI 1-3, subframe index and amp; expected: the
REG mapping and the digest of symbol 0 of that subframe per antenna.

Each modulation case: a frame (N_RB_DL, Ncp, TX antennas, mode1_flag, Nid_cell), a transmission
mode (SISO / ALAMOUTI / LARGE_CDD, one or two codewords), the subframe index, PDCCH symbols, an RB
bitmap, amp and rho_A / rho_B; expected: dlsch_modulation's return value and the digest of each
antenna's subframe of the frame grid."""
import numpy as np

from rm_ref_cases import digest, splitmix64

NBITS = 14 * 1200 * 6
FULL = {6: (0x3F, 0, 0, 0), 15: (0x7FFF, 0, 0, 0), 25: (0x1FFFFFF, 0, 0, 0), 50: (0xFFFFFFFF, 0x3FFFF, 0, 0),
        100: (0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xF)}


def e_bits(seed):
    """NBITS entries 0/1: the bits of splitmix64(seed) words, LSB first."""
    w = splitmix64(seed, NBITS // 64 + 1)
    return np.unpackbits(w.view(np.uint8), bitorder="little")[:NBITS].astype(np.uint8)


def alloc_bits(seed, n_rb):
    """a sparse RB bitmap (about a quarter of the RBs, never empty)"""
    w = splitmix64(seed ^ 0xA11C, 4)
    m = 0
    for i in range(n_rb):
        if (int(w[i % 4]) >> (i // 4 * 3 % 61)) & 3 == 0:
            m |= 1 << i
    m |= 1 << (n_rb // 2)
    return tuple((m >> (32 * i)) & 0xFFFFFFFF for i in range(4))


def modulation_cases():
    cases = []
    k = 0
    for n_rb in (6, 15, 25, 50, 100):
        for mode, n_ant, n_cw, mode1 in ((0, 1, 1, 1), (0, 2, 1, 1), (1, 2, 1, 0), (2, 2, 2, 0)):
            for sf in (0, 5, 7):
                k += 1
                mcs = [(5, 12, 22, 19)[(k + c) % 4] for c in range(n_cw)]
                cases.append(dict(N_RB_DL=n_rb, Ncp=1 if (k % 5 == 0) else 0, n_ant=n_ant, mode1_flag=mode1,
                                  Nid_cell=(37 * k) % 504, mimo_mode=mode, n_cw=n_cw, mcs=mcs, subframe=sf,
                                  num_pdcch=(1, 2, 3)[k % 3] if n_rb > 10 else (2, 3, 4)[k % 3],
                                  rb_alloc=list(FULL[n_rb] if k % 4 else alloc_bits(k, n_rb)),
                                  amp=512, rho=[(8192, 8192), (5793, 8192), (8192, 11585)][k % 3] if mode == 1
                                  else (8192, 8192), seed=[0x30D0000 + 16 * k + c for c in range(n_cw)]))
    # the C3 subframe itself
    cases.append(dict(N_RB_DL=100, Ncp=0, n_ant=2, mode1_flag=0, Nid_cell=0, mimo_mode=2, n_cw=2, mcs=[19, 19],
                      subframe=7, num_pdcch=1, rb_alloc=list(FULL[100]), amp=512, rho=(8192, 8192),
                      seed=[0x3C30000, 0x3C30001]))
    return cases


def scrambling_cases():
    return [dict(G=G, rnti=rnti, Nid_cell=nid, q=q, Ns=Ns, seed=0x5C00000 + i)
            for i, (G, rnti, nid, q, Ns) in enumerate([(1512, 0x1234, 0, 0, 14), (60000, 0x1234, 0, 0, 14),
                                                       (86400, 0x1234, 0, 1, 14), (86400, 0xFFFF, 503, 0, 0),
                                                       (33, 1, 37, 1, 19), (14400, 0x8000, 255, 0, 10)])]


def grid_digests(grids, c, N):
    """per-antenna digests of subframe c["subframe"] of frame grids"""
    nsymb = 12 if c["Ncp"] else 14
    sf = c["subframe"]
    return [digest(g[sf * nsymb * N:(sf + 1) * nsymb * N]) for g in grids]


def cws_of(c):
    return [dict(e=e_bits(c["seed"][i]), mcs=c["mcs"][i], mimo_mode=c["mimo_mode"], rb_alloc=c["rb_alloc"])
            for i in range(c["n_cw"])]


def frame_of(O, c):
    return O.frame(c["N_RB_DL"], Nid_cell=c["Nid_cell"], Ncp=c["Ncp"], nb_antennas_tx=c["n_ant"],
                   mode1_flag=c["mode1_flag"])


def pcfich_cases():
    """every bandwidth, both prefixes, 1 TX antenna (SISO), 2 (SISO and ALAMOUTI), CFI 1-3"""
    cases = []
    k = 0
    for n_rb in (6, 15, 25, 50, 100):
        for n_ant, mode1 in ((1, 1), (2, 1), (2, 0)):
            for cfi in (1, 2, 3):
                k += 1
                cases.append(dict(N_RB_DL=n_rb, Ncp=1 if k % 4 == 0 else 0, n_ant=n_ant, mode1_flag=mode1,
                                  Nid_cell=(97 * k + 11) % 504, cfi=cfi, subframe=(3 * k) % 10,
                                  amp=(512, 1024, 4096, 32767)[k % 4]))
    return cases


def symbol0_digests(grids, c, N):
    """per-antenna digests of symbol 0 of subframe c["subframe"] of frame grids"""
    nsymb = 12 if c["Ncp"] else 14
    o = c["subframe"] * nsymb * N
    return [digest(g[o:o + N]) for g in grids]
