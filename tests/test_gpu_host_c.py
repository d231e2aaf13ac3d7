"""The C host drivers (tools/dlsim_tx.c, tools/dlsim_rx.c; gcc, linked against libopenair4g_amd.so) on the GPU:
dlsim's transmit loop through the drop-in entry points and through oai4g_tx_batch.  The IQ of
both equals the committed golden vectors (C3 digest, C1 samples) and each other."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tools", "bin", "dlsim_tx")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _run(tmp_path, cfg, sf, pays, batch=64):
    pf = tmp_path / "pay.bin"
    pf.write_bytes(b"".join(np.ascontiguousarray(p).tobytes() for p in pays))
    r = subprocess.run([EXE, "-c", cfg, "-s", str(sf), "-n", "3", "-B", str(batch), "-i", str(pf),
                        "-o", str(tmp_path / "drop.bin"), "-O", str(tmp_path / "batch.bin"), "-P"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Total PHY proc tx" in r.stdout
    return (tmp_path / "drop.bin").read_bytes(), (tmp_path / "batch.bin").read_bytes()


def test_dlsim_tx_c3_matches_golden(gpu, tmp_path):
    row = json.load(open(os.path.join(GOLDEN, "pipeline_C3.json")))["subframes"][0]
    assert row["subframe"] == 7
    rng = np.random.default_rng(33)
    p = gpu.make_params("C3", subframe=7)
    pays = [rng.integers(0, 256, size=p.TBS[cw] // 8, dtype=np.uint8) for cw in range(p.n_cw)]
    drop, batch = _run(tmp_path, "C3", 7, pays)
    assert hashlib.sha256(drop).hexdigest() == row["iq_sha256"]
    assert drop == batch


def test_dlsim_tx_c1_matches_golden(gpu, tmp_path):
    z = np.load(os.path.join(GOLDEN, "pipeline_C1.npz"))
    for sf in (0, 5, 7):
        drop, batch = _run(tmp_path, "C1", sf, [z[f"payload0_{sf}"]])
        assert np.array_equal(np.frombuffer(drop, np.int32).reshape(z[f"iq_{sf}"].shape), z[f"iq_{sf}"]), sf
        assert drop == batch


@pytest.mark.parametrize("cfg", ["C2", "TM2"])
def test_dlsim_tx_drop_in_equals_batch(gpu, tmp_path, cfg):
    p = gpu.make_params(cfg, subframe=5)
    rng = np.random.default_rng(9)
    pays = [rng.integers(0, 256, size=p.TBS[cw] // 8, dtype=np.uint8) for cw in range(p.n_cw)]
    drop, batch = _run(tmp_path, cfg, 5, pays)
    assert drop == batch


RX_EXE = os.path.join(ROOT, "tools", "bin", "dlsim_rx")


@pytest.mark.parametrize("nrb,mcs,npd,sf,n", [(100, 16, 1, 1, 4), (100, 27, 2, 6, 3), (50, 9, 3, 7, 3),
                                             (25, 16, 1, 1, 4), (6, 9, 3, 2, 3)])
def test_dlsim_rx_closes_the_downlink_loop_in_c(gpu, nrb, mcs, npd, sf, n):
    """tools/dlsim_rx.c: the whole dlsim loop from C over the device API (tx batch -> FEP -> channel
    estimation -> frequency offset / time-domain estimate -> rx_pdsch -> dlsch_decoding chain): every
    transport block comes back bit-exact.  With the identity channel the frequency-offset estimate is
    the reference arithmetic's own bias (the per-RE floor of ">> dl_ch_shift": about -34 Hz, see
    tests/test_freq_offset_cpu.py) and the timing tracker's peak sits at the first samples."""
    r = subprocess.run([RX_EXE, "-r", str(nrb), "-m", str(mcs), "-p", str(npd), "-s", str(sf), "-n", str(n), "-P"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all transport blocks recovered" in r.stdout
    import re
    f = int(re.search(r"freq_offset (-?\d+) Hz", r.stdout).group(1))
    peak = int(re.search(r"timing peak (\d+)", r.stdout).group(1))
    assert abs(f) < 60 and peak <= 4, r.stdout


def test_dlsim_rx_refuses_subframes_0_and_5(gpu):
    r = subprocess.run([RX_EXE, "-s", "4", "-n", "2"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "0 / 5" in r.stderr
