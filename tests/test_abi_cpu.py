"""CPU suite: the drop-in C ABI (include/oai4g.h) and the host-side mirror, without a GPU.

  - the shared library loads and exports every function include/oai4g.h declares;
  - the Python mirror binds every export, and its ctypes struct layouts equal the C layouts
    (sizes and offsets from a tiny C program compiled against the header);
  - without a gfx950 device the library refuses to run (no CPU fallback): oai4g_init() < 0;
  - host-side helpers (frame parameters, G, Gold) agree with the oracle.
"""
import ctypes
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_lib as O
import openair4g_amd as oai

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "oai4g.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(oai4g_\w+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    return oai.load_library()


def test_library_exports_every_declared_function(lib):
    names = header_functions()
    assert len(names) > 40
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_python_mirror_binds_every_export():
    assert set(header_functions()) <= set(oai.exported_symbols())


def test_no_reference_or_oracle_symbols_in_product():
    """The product library must not contain (or route through) the CPU oracle."""
    out = subprocess.run(["nm", "-D", "--defined-only", oai.LIB_PATH], capture_output=True, text=True).stdout
    assert "orc_" not in out


def _c_layout(struct, fields):
    src = "#include <stdio.h>\n#include <stddef.h>\n#include \"oai4g.h\"\nint main(void){\n"
    src += f'printf("%zu\\n", sizeof({struct}));\n'
    for f in fields:
        src += f'printf("%zu\\n", offsetof({struct}, {f}));\n'
    src += "return 0;}\n"
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        exe = os.path.join(d, "l")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        vals = [int(v) for v in subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()]
    return vals[0], vals[1:]


@pytest.mark.parametrize("cls,cname", [(oai.TxParams, "oai4g_tx_params_t"), (oai.FrameParms, "oai4g_frame_parms_t")])
def test_struct_layouts_match_header(cls, cname):
    fields = [f[0] for f in cls._fields_ if not f[0].startswith("_")]
    size, offs = _c_layout(cname, fields)
    assert ctypes.sizeof(cls) == size
    assert [getattr(cls, f).offset for f in fields] == offs


def test_init_without_gpu_fails_loudly(lib):
    rc = lib.oai4g_init()
    if rc == 0:
        pytest.skip("a gfx950 device is present (this check is for GPU-less hosts)")
    assert rc < 0
    assert lib.oai4g_last_error()
    with pytest.raises(oai.OAI4GError):
        oai.init()


def test_frame_parms_match_oracle(lib):
    for N_RB in (6, 15, 25, 50, 100):
        fp = oai.FrameParms()
        assert lib.oai4g_init_frame_parms(ctypes.byref(fp), N_RB, 3, 0, 2, 0, 0) == 0
        ref = O.frame(N_RB, 3, 0, 2, 0, 0)
        for f in ("ofdm_symbol_size", "first_carrier_offset", "nb_prefix_samples", "nb_prefix_samples0",
                  "samples_per_tti", "nushift", "symbols_per_tti"):
            assert getattr(fp, f) == getattr(ref, f), (N_RB, f)


def test_get_G_and_Qm_match_oracle(lib):
    rng = np.random.default_rng(5)
    for _ in range(60):
        N_RB = int(rng.choice([6, 15, 25, 50, 100]))
        mode1 = int(rng.integers(0, 2))
        fp = oai.FrameParms()
        lib.oai4g_init_frame_parms(ctypes.byref(fp), N_RB, 0, 0, 1 if mode1 else 2, mode1, 0)
        alloc = [int(v) for v in rng.integers(0, 2 ** 32, 4, dtype=np.uint64)]
        alloc[3] &= 0xF
        nb_rb = sum(bin(a).count("1") for a in alloc[:((N_RB + 31) // 32)])
        mcs, pdcch, sf = int(rng.integers(0, 29)), int(rng.integers(1, 4)), int(rng.integers(0, 10))
        Qm = lib.oai4g_get_Qm(mcs)
        assert Qm == O.orc().orc_get_Qm(mcs)
        ra = (ctypes.c_uint32 * 4)(*alloc)
        g = lib.oai4g_get_G(ctypes.byref(fp), nb_rb, ra, Qm, 1, pdcch, 0, sf)
        assert g == O.get_G(N_RB, 0, mode1, 0, nb_rb, alloc, Qm, 1, pdcch, sf)


def test_gold_generic_matches_oracle(lib):
    for c_init in (1, 0x1234 << 14 | 5 << 9 | 7, 0x5A5A5A5):
        a1, a2 = ctypes.c_uint32(0), ctypes.c_uint32(c_init)
        b1, b2 = ctypes.c_uint32(0), ctypes.c_uint32(c_init)
        for i in range(20):
            assert lib.oai4g_lte_gold_generic(ctypes.byref(a1), ctypes.byref(a2), int(i == 0)) == \
                O.orc().orc_gold_generic(ctypes.byref(b1), ctypes.byref(b2), int(i == 0))


def test_params_block_round_trip():
    for name, tbs in (("C1", [936]), ("C2", [30576]), ("C3", [36696, 36696])):
        p = oai.make_params(name, subframe=5, subframe_step=1)
        q = oai.TxParams.from_bytes(p.to_bytes())
        assert q.to_bytes() == p.to_bytes()
        assert [q.TBS[i] for i in range(q.n_cw)] == tbs
