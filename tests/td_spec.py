"""Textbook turbo decoder — TEST INFRASTRUCTURE ONLY.

An independent model of the 36.212 5.1.3.2 parallel-concatenated code's iterative decoder,
written from the BCJR / max-log-MAP definition (Bahl et al.; Robertson, Villebrun & Hoeher),
not from the reference's SSE schedule: floating point, whole-block forward/backward recursions
(no windows), trellis termination of both constituent codes, extrinsic exchange through the
QPP interleaver, a fixed number of full iterations, hard decision on the a-posteriori LLR.

It pins the oracle decoder (oracle/oai_oracle_td.c, a restatement of
3gpplte_turbo_decoder_sse_16bit.c whose translation unit cannot be built here) where the two
must agree whatever their arithmetic: every block the oracle reports as CRC-passing must be the
block this model decodes.

Input layout = the reference's decoder input (3gpplte_turbo_decoder_sse_16bit.c:945-1000):
(x_k, z_k, z'_k) for k < K, then x_K z_K x_K+1 z_K+1 x_K+2 z_K+2 x'_K z'_K ... (the tail of
tests/spec_model.turbo_encode); positive = bit 1.
"""
import numpy as np


def _trellis():
    """8-state RSC g0 = 1 + D^2 + D^3, g1 = 1 + D + D^3 (36.212 5.1.3.2.1).
    state = d1 + 2 d2 + 4 d3 (shift-register contents)."""
    nxt = np.zeros((8, 2), np.int64)
    par = np.zeros((8, 2), np.int64)
    for s in range(8):
        d1, d2, d3 = s & 1, (s >> 1) & 1, (s >> 2) & 1
        for u in range(2):
            a = u ^ d2 ^ d3
            par[s, u] = a ^ d1 ^ d3
            nxt[s, u] = a | (d1 << 1) | (d2 << 2)
    # the two predecessors (state, input) of every state
    pred = [[] for _ in range(8)]
    for s in range(8):
        for u in range(2):
            pred[nxt[s, u]].append((s, u))
    ps = np.array([[p[0][0], p[1][0]] for p in pred])
    pu = np.array([[p[0][1], p[1][1]] for p in pred])
    # termination: input = feedback (a = 0), tail systematic bit x = d2 ^ d3, parity d1 ^ d3
    tnext = np.array([((s & 1) << 1) | (((s >> 1) & 1) << 2) for s in range(8)])
    tx = np.array([((s >> 1) ^ (s >> 2)) & 1 for s in range(8)])
    tz = np.array([(s ^ (s >> 2)) & 1 for s in range(8)])
    return nxt, par, ps, pu, tnext, tx, tz


NXT, PAR, PS, PU, TNEXT, TX, TZ = _trellis()
NEG = -1e30


def _siso(Ls, Lp, La, tail_x, tail_z):
    """Max-log-MAP of one constituent code, batched over blocks.
    Ls, Lp, La: [B, K] channel systematic, channel parity, a-priori LLRs; tail_*: [B, 3].
    Returns the a-posteriori LLR [B, K]."""
    B, K = Ls.shape
    sgn = np.array([-1.0, 1.0])
    # branch metric of (state s, input u) at step k: 0.5 (u~ (Ls + La) + p~ Lp)
    Lu = 0.5 * (Ls + La)
    Lq = 0.5 * Lp
    gam_p = (sgn[PU][None, None, :, :] * Lu[:, :, None, None] +
             sgn[PAR[PS, PU]][None, None, :, :] * Lq[:, :, None, None])   # [B, K, 8, 2] for pred pairs
    alpha = np.empty((K + 1, B, 8))
    a = np.full((B, 8), NEG)
    a[:, 0] = 0.0
    alpha[0] = a
    for k in range(K):
        a = np.max(a[:, PS] + gam_p[:, k], axis=2)
        a -= a.max(axis=1, keepdims=True)
        alpha[k + 1] = a
    # tail (3 forced steps) backward from state 0
    b = np.full((B, 8), NEG)
    b[:, 0] = 0.0
    for t in (2, 1, 0):
        g = 0.5 * (sgn[TX][None, :] * tail_x[:, t:t + 1] + sgn[TZ][None, :] * tail_z[:, t:t + 1])
        b = b[:, TNEXT] + g
    b -= b.max(axis=1, keepdims=True)
    # backward over the data, with the a-posteriori LLR of each step
    gam_f = sgn[np.arange(2)][None, None, None, :] * Lu[:, :, None, None] + \
        sgn[PAR][None, None, :, :] * Lq[:, :, None, None]                 # [B, K, 8(s), 2(u)]
    app = np.empty((B, K))
    for k in range(K - 1, -1, -1):
        m = alpha[k][:, :, None] + gam_f[:, k] + b[:, NXT]                  # [B, 8, 2]
        app[:, k] = m[:, :, 1].max(axis=1) - m[:, :, 0].max(axis=1)
        b = np.max(gam_f[:, k] + b[:, NXT], axis=2)
        b -= b.max(axis=1, keepdims=True)
    return app


def decode(y, K, f1, f2, iterations=8):
    """y: [B, 3K+12] LLRs (positive = 1).  Returns hard decisions [B, K] (0/1) after `iterations`
    full iterations (decoder 1 then decoder 2 each)."""
    y = np.atleast_2d(np.asarray(y, dtype=np.float64))
    B = y.shape[0]
    pi = (f1 * np.arange(K, dtype=np.int64) + f2 * np.arange(K, dtype=np.int64) ** 2) % K
    xs, z1, z2 = y[:, 0:3 * K:3], y[:, 1:3 * K:3], y[:, 2:3 * K:3]
    t = y[:, 3 * K:]
    tx1, tz1 = t[:, 0:6:2], t[:, 1:6:2]
    tx2, tz2 = t[:, 6:12:2], t[:, 7:12:2]
    xs_i = xs[:, pi]
    Le2 = np.zeros((B, K))           # extrinsic of decoder 2, de-interleaved
    app2 = np.zeros((B, K))
    for _ in range(iterations):
        app1 = _siso(xs, z1, Le2, tx1, tz1)
        Le1 = app1 - xs - Le2
        La2 = Le1[:, pi]
        app2 = _siso(xs_i, z2, La2, tx2, tz2)
        Le2i = app2 - xs_i - La2
        Le2 = np.empty_like(Le2i)
        Le2[:, pi] = Le2i
    L = np.empty_like(app2)
    L[:, pi] = app2
    return (L > 0).astype(np.uint8)


def bits_to_bytes(bits):
    """MSB-first packing (the decoder output layout, bit k = bit 7 - k%8 of byte k/8)."""
    return np.packbits(np.asarray(bits, dtype=np.uint8), axis=-1)
