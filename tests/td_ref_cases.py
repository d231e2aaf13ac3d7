"""Turbo-encoder pin through the reference's own scalar decoder (oracle/_ref/libref_td.so:
PHY/CODING/3gpplte_turbo_decoder.c, phy_threegpplte_turbo_decoder_scalar :883, compiled unmodified).
TEST INFRASTRUCTURE, shared by tests/test_ref_pin_td_cpu.py (live, build container),
tests/test_td_ref_fixture_cpu.py (fixture, anywhere), tests/test_gpu_td_ref.py (GPU) and
tests/golden/gen_td_ref.py (writes tests/golden/td_ref.json).

The reference encoder TU (3gpplte_sse.c) cannot be built (its QPP tables live in the missing blob
lte_interleaver.h), but this decoder walks Π with the closed-form recursion of
lte_interleaver_inline.h:38-51 and carries the RSC in its branch-metric tables (:63-82).  A codeword it
decodes back to the encoder's input, with the CRC the decoder checks (:1023-1072) passing, is
reference-executed evidence for the encoder's RSC and QPP order.  Noiseless ±AMP LLRs alone would
decode from the systematic stream, so the variants take it away:

  full     every stream;
  nosys    systematic LLRs (x_k, and the x / x' of the tails) zeroed: the decision rests on z and z';
  z_only   nosys with z' zeroed too: encoder 1 (the RSC) alone must carry the block;
  zp_only  nosys with z zeroed: encoder 2 (QPP order + RSC) alone must carry the block;
  flip     AMP_FLIP, full streams, 3 % of the systematic LLRs sign-flipped at seeded positions: the
           parity streams must correct them.
Negative controls: nosys / zp_only decoded with the (f1, f2) of the next K in Table 5.1.3-3 must fail.

What this decoder cannot pin: the trellis tails (d[3K .. 3K+11]).  Its termination code is commented
out (:583-672; beta starts from alpha at K, :674-681) and the second encoder's tail read indexes past
the tail (:1001-1003, systematic0[i + 8]), so no tail LLR reaches a decision.  The tails stay pinned
to the 36.212 spec model (tests/spec_model.py) only.

Two reference overruns shape the cases (both in the unmodified TU, both measured here):
  - compute_ext_s writes ext[0 .. K+2] (:819-873) into the VLAs `short ext[n], ext2[n]` (:895).  K is a
    multiple of 8, so the VLAs have no padding: ext2's 3 extra entries land on ext[0..2] (rewritten
    before they are read) and ext's on the lowest slot of the fixed frame.  In this build (gcc 11.4 -O2,
    objdump of _ref/3gpplte_turbo_decoder.o) that slot holds the CRC24_A argument &decoded_bytes[F >> 3]
    (:1032), read from the second iteration on: a CRC24_A block that does not decode at iteration 1
    segfaults.  The CRC24_B path never reads the slot, so every case here uses CRC24_B (crc_type 1), the
    CRC every block of a multi-block transport block carries (C3: C = 6).
  - the globals hold 6144 entries (:355) but the tail copies write systematic0[K .. K+5], yparity1/2[K ..
    K+2] and systematic2[K .. K+2] (:945-958, :1001-1003).  At K = 6144 these land in the next .bss
    object (nm -n: beta, alpha, cpu_freq_GHz, systematic0): systematic2's overrun rewrites
    systematic0[0..2] with stale beta values every iteration.  The K = 6144 row still decodes every variant.
Calls are serial (one process, one thread): the decoder's state is global."""
import hashlib

import numpy as np

import oracle_lib as O
from ref_cases import QPP, crc_block

AMP = 4                 # ≤ 8: above it the 16-bit metrics saturate on long blocks and nosys fails (K ≥ 1120 at 64)
AMP_FLIP = 2
FLIP_FRAC = 0.03
MAX_IT = 8
KS = tuple(sorted(QPP))
VARIANTS = ("full", "nosys", "z_only", "zp_only", "flip")
NEG_VARIANTS = ("nosys", "zp_only")
SEED = 0x7D0


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def neighbour(K):
    i = KS.index(K)
    return KS[i + 1] if i + 1 < len(KS) else KS[i - 1]


def blocks():
    """(K, crc_type, c): one CRC24_B-terminated block per Table 5.1.3-3 size, seeded (crc_type 1; the
    module docstring says why not CRC24_A)."""
    rng = np.random.default_rng(SEED)
    return [(K, 1, crc_block(rng, K, 1)) for K in KS]


def flip_positions(K, salt=0):
    rng = np.random.default_rng((SEED << 16) + (K << 2) + salt)
    return rng.choice(K, int(FLIP_FRAC * K), replace=False) * 3


def sys_positions(K):
    """x_k (k < K) and the systematic entries of both tails (d[3K + 2j], j < 6)."""
    return np.concatenate([np.arange(0, 3 * K, 3), 3 * K + 2 * np.arange(6)])


def variant(d, K, name):
    """int16 LLRs (positive = bit 1, :1019) of the 3K+12 entry d in the decoder's read order."""
    d = np.asarray(d[:3 * K + 12], np.int16)
    if name == "flip":
        y = (d * 2 - 1) * AMP_FLIP
        p = flip_positions(K)
        y[p] = -y[p]
        return y.astype(np.int16)
    y = ((d * 2 - 1) * AMP).astype(np.int16)
    if name == "full":
        return y
    y[sys_positions(K)] = 0
    if name == "z_only":
        y[2:3 * K:3] = 0
        y[3 * K + 6 + 1::2] = 0          # z' of the second tail
    elif name == "zp_only":
        y[1:3 * K:3] = 0
        y[3 * K + 1:3 * K + 6:2] = 0     # z of the first tail
    return y


def decode(y, K, crc_type, qpp=None):
    f1, f2 = QPP[K] if qpp is None else qpp
    return O.ref_turbo_decode_scalar(y, K, f1, f2, MAX_IT, crc_type, 0)


def check_block(d, K, crc_type, c):
    """Every variant decodes to c with the CRC passing; the negative controls fail.  Returns the
    fixture row {variant: [iterations, digest(decoded)]}."""
    row = {}
    for v in VARIANTS:
        it, dec = decode(variant(d, K, v), K, crc_type)
        assert it <= MAX_IT and np.array_equal(dec, c), (K, v, it)
        row[v] = [it, digest(dec)]
    for v in NEG_VARIANTS:
        it, dec = decode(variant(d, K, v), K, crc_type, QPP[neighbour(K)])
        assert it == MAX_IT + 1 and not np.array_equal(dec, c), (K, "neg", v, it)
        row["neg_" + v] = [it, digest(dec)]
    return row


# ---- receive side of a whole codeword, reference functions only (C3 / C2 bench blocks) ----
def rx_block_llrs(ebits_cw, G, C, r, K, Qm, Kmimo, Nl, gold_bits, amp=AMP_FLIP):
    """Descramble the codeword's e bits with the reference's Gold bits, map to ±amp soft bits, and run
    the reference's lte_rate_matching_turbo_rx (lte_rate_matching.c:688) and
    sub_block_deinterleaving_turbo (:193) for block r: the decoder-order int16 LLRs of d."""
    D = K + 4
    R = (D + 31) >> 5
    bits = (np.asarray(ebits_cw[:G], np.uint8) & 1) ^ gold_bits[:G]
    soft = ((bits.astype(np.int16) * 2 - 1) * amp).astype(np.int16)
    Qb = Nl * Qm
    Gp = G // Qb
    gamma = Gp % C
    E = [Qb * (Gp // C) if i <= C - gamma - 1 else Qb * -(-Gp // C) for i in range(C)]   # :523-533
    off = sum(E[:r])
    _, dw = O.ref_dummy_w(D)
    ret, Er, w = O.ref_rate_match_rx(R, G, np.zeros(3 * 32 * R, np.int16), dw, soft[off:], C, r, Qm, clear=1,
                                     Nl=Nl, Kmimo=Kmimo)
    assert ret == 0 and Er == E[r], (ret, Er, E[r])
    return O.ref_deinterleave(D, w)[96:96 + 3 * K + 12].copy()


def decode_codeword(ebits, G, K, C, Qm, Kmimo, Nl, gold_bits, tbs):
    """A whole scrambled codeword (G e bits of one transport block, F = 0 and every block K, as C2 / C3
    segment) received with reference functions only: rx_block_llrs per block, 3 % of the systematic
    LLRs sign-flipped (flip_positions, salted by r), phy_threegpplte_turbo_decoder_scalar with CRC24_B.
    Returns (per-block iteration counts, the transport block bytes the blocks carry: TBS/8 payload
    bytes then the 3 CRC24_A bytes)."""
    its, parts = [], []
    for r in range(C):
        y = rx_block_llrs(ebits, G, C, r, K, Qm, Kmimo, Nl, gold_bits)
        p = flip_positions(K, salt=r + 1)
        y[p] = -y[p]
        it, dec = decode(y, K, 1)
        its.append(it)
        parts.append(dec[:(K - 24) // 8])
    tb = np.concatenate(parts)
    assert len(tb) == tbs // 8 + 3
    return its, tb
