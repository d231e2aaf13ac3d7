"""The reference-side shim (integration/oai4g_shim.c) must export each reference function under its
own name with the reference's own parameter types, so a dlsim linked with it resolves every call
to the GPU binding with no other change.  Checked here against the prototypes in the reference's
headers (PHY/**/*.h, or the defining .c file when no header declares it; read as text, when the
reference tree is present): the
return type (exactly) and every parameter type, after normalising whitespace, parameter names and the
`const` the reference omits.  (oai4g_shim.c also compiles and runs against the reference's headers: tests/test_gpu_shim_ref.py; the
PHY_VARS_* bindings of oai4g_shim_ue.c need the asn1c-generated headers to compile, so
this is the check of the boundary that runs here; test_integration_cpu.py checks the oai4g_ side.)"""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/openair1"
SHIM = os.path.join(ROOT, "integration", "oai4g_shim.c")
SHIM_UE = os.path.join(ROOT, "integration", "oai4g_shim_ue.c")    # the PHY_VARS_* bindings

# other spellings of the same types (module_id_t: openair2/COMMON/platform_types.h:70; the header
# declares lte_dl_channel_estimation's eNB_id as module_id_t, its definition as uint8_t)
TYPE_ALIASES = {"module_id_t": "uint8_t", "short": "int16_t", "unsigned short": "uint16_t", "unsigned char": "uint8_t", "int": "int32_t",
                "unsigned int": "uint32_t", "signed char": "int8_t"}
# plain `char` is a distinct C type (neither int8_t nor uint8_t): it is deliberately not aliased


def _strip(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _norm_type(t):
    t = " ".join(t.replace("*", " * ").split())
    t = re.sub(r"\bconst\b", "", t)
    t = " ".join(t.split())
    base = t.replace(" *", "").strip()
    stars = t.count("*")
    base = TYPE_ALIASES.get(base, base)
    return base + "*" * stars


def _params(args):
    args = " ".join(args.split())
    if args in ("", "void"):
        return []
    out = []
    for a in args.split(","):
        a = a.strip()
        m = re.match(r"(.*?)(\w+)\s*(\[\s*\w*\s*\])?$", a)
        typ, arr = (m.group(1), m.group(3)) if m and m.group(1).strip() else (a, None)
        out.append(_norm_type(typ + (" *" if arr else "")))
    return out


def _shim_functions():
    s = _strip(open(SHIM).read() + "\n" + open(SHIM_UE).read())
    fns = {}
    for ret, name, args in re.findall(r"^(?!static)([A-Za-z_][\w \*]*?)\b(\w+)\(([^;{]*?)\)\s*\{", s, flags=re.M):
        fns[name] = (_norm_type(ret), _params(args))
    return fns


def _ref_prototypes(names):
    found = {}
    files = glob.glob(os.path.join(REF, "PHY", "**", "*.h"), recursive=True)
    for f in files:
        try:
            txt = _strip(open(f, errors="replace").read())
        except OSError:
            continue
        for name in names:
            if name in found:
                continue
            m = re.search(r"(?:^|[;}\n])\s*(?:extern\s+)?([A-Za-z_][\w \*]*?)\b" + re.escape(name) + r"\s*\(([^;{)]*)\)\s*;",
                          txt)
            if m:
                found[name] = (_norm_type(m.group(1)), _params(m.group(2)), os.path.relpath(f, REF))
    # functions the reference declares nowhere but defines in its .c file (generate_phich): the definition
    for f in glob.glob(os.path.join(REF, "PHY", "**", "*.c"), recursive=True):
        if all(n in found for n in names):
            break
        try:
            txt = _strip(open(f, errors="replace").read())
        except OSError:
            continue
        for name in names:
            if name in found:
                continue
            m = re.search(r"(?:^|\n)([A-Za-z_][\w \*]*?)\b" + re.escape(name) + r"\s*\(([^;{)]*)\)\s*\{", txt)
            if m:
                found[name] = (_norm_type(m.group(1)), _params(m.group(2)), os.path.relpath(f, REF))
    return found


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree absent")
def test_shim_signatures_equal_reference_prototypes():
    shim = _shim_functions()
    assert len(shim) >= 40
    ref = _ref_prototypes(list(shim))
    # bound by name from a reference declaration; every binding must find one
    missing = sorted(set(shim) - set(ref))
    assert not missing, f"no reference prototype found for {missing}"
    bad = []
    for name, (ret, params) in shim.items():
        rret, rparams, where = ref[name]
        if params != rparams or ret != rret:
            bad.append((name, where, (ret, params), (rret, rparams)))
    assert not bad, "\n".join(map(str, bad))


def test_normaliser_keeps_distinct_types_distinct():
    """The comparison would catch the prototype mismatches a lenient check lets through."""
    assert _norm_type("char *") != _norm_type("int8_t *")
    assert _norm_type("char") != _norm_type("uint8_t")
    assert _norm_type("int") != _norm_type("uint32_t")
    assert _norm_type("int32_t") != _norm_type("int16_t")
    assert _norm_type("unsigned char") == _norm_type("uint8_t")
    assert _norm_type("const short *") == _norm_type("int16_t*")
    assert _params("uint8_t *a, int b[2], LTE_DL_FRAME_PARMS *fp") == ["uint8_t*", "int32_t*", "LTE_DL_FRAME_PARMS*"]
