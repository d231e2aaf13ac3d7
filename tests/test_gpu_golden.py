"""GPU parity against the committed golden fixtures (tests/golden/, see gen_golden.py):
the reference's own IDFT outputs, and the C1 / C3 transmit vectors.  Bit-exact."""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_gpu_idft_matches_reference_outputs(gpu):
    z = np.load(os.path.join(GOLDEN, "idft_ref.npz"))
    n = 0
    for key in z.files:
        if key.startswith("x_"):
            _, size, vi, scale = key.split("_")
            assert np.array_equal(gpu.idft(z[key], int(scale)), z[f"y_{size}_{vi}_{scale}"]), key
            n += 1
    assert n == 24


def _run_one(gpu, p, pays):
    pipe = gpu.TxPipeline(p, 1)
    buf = np.zeros((1, p.n_cw, p.payload_stride), dtype=np.uint8)
    for cw, pl in enumerate(pays):
        buf[0, cw, :len(pl)] = pl
    pipe.upload_payload(buf)
    pipe.run()
    pipe.sync()
    iq, eb = pipe.iq()[0].copy(), pipe.ebits()[0].copy()
    Gs = [pipe.G(cw, p.first_subframe) for cw in range(p.n_cw)]
    pipe.close()
    ebits = [np.packbits(gpu.unpack_bits(eb[cw], Gs[cw]), bitorder="little") for cw in range(p.n_cw)]
    return iq, ebits


def test_gpu_matches_c1_fixture(gpu):
    z = np.load(os.path.join(GOLDEN, "pipeline_C1.npz"))
    for sf in (0, 5, 7):
        p = gpu.make_params("C1", subframe=sf)
        iq, ebits = _run_one(gpu, p, [z[f"payload0_{sf}"]])
        assert np.array_equal(ebits[0], z[f"ebits0_{sf}"]), sf
        assert np.array_equal(iq, z[f"iq_{sf}"]), sf


def test_gpu_matches_c3_fixture(gpu):
    fx = json.load(open(os.path.join(GOLDEN, "pipeline_C3.json")))
    rng = np.random.default_rng(33)
    for row in fx["subframes"]:
        sf = row["subframe"]
        p = gpu.make_params("C3", subframe=sf)
        pays = [rng.integers(0, 256, size=p.TBS[cw] // 8, dtype=np.uint8) for cw in range(p.n_cw)]
        assert [hashlib.sha256(pl.tobytes()).hexdigest() for pl in pays] == row["payload_sha256"]
        iq, ebits = _run_one(gpu, p, pays)
        assert [hashlib.sha256(e.tobytes()).hexdigest() for e in ebits] == row["ebits_sha256"], sf
        assert iq[:, :16].tolist() == row["iq_head"], sf
        assert hashlib.sha256(np.ascontiguousarray(iq).tobytes()).hexdigest() == row["iq_sha256"], sf


def test_gpu_pipelined_batch_equals_serial(gpu, monkeypatch):
    """The optional two-stream chunked batch (OAI4G_PIPE_CHUNK) produces the serial result."""
    p = gpu.make_params("C3", subframe=0, subframe_step=1)
    n_sf = 40
    rng = np.random.default_rng(4)
    pay = rng.integers(0, 256, size=(n_sf, p.n_cw, p.payload_stride), dtype=np.uint8)
    out = []
    for chunk in ("0", "8"):
        monkeypatch.setenv("OAI4G_PIPE_CHUNK", chunk)
        pipe = gpu.TxPipeline(p, n_sf)
        pipe.upload_payload(pay)
        pipe.run()
        pipe.sync()
        out.append(pipe.iq().copy())
        pipe.close()
    assert np.array_equal(out[0], out[1])
