"""The reference-side shim (integration/oai4g_shim.c) and the C host driver
(tools/dlsim_tx.c) against the C ABI: every oai4g_ entry point they call is declared in
include/oai4g.h with the same number of arguments and exported by the built library; the C
driver compiles with gcc -Wall -Werror against the header alone."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = open(os.path.join(ROOT, "include", "oai4g.h")).read()


def _strip_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _calls(src):
    """{name: n_args} of every `oai4g_name(` call / declaration in src (top-level commas)."""
    out = {}
    for m in re.finditer(r"\boai4g_(\w+)\s*\(", src):
        i, depth, args, cur = m.end(), 1, [], ""
        while depth:
            ch = src[i]
            if ch == "(":
                depth += 1
            elif ch == ")":
                depth -= 1
                if depth == 0:
                    break
            if ch == "," and depth == 1:
                args.append(cur)
                cur = ""
            else:
                cur += ch
            i += 1
        args.append(cur)
        n = 0 if len(args) == 1 and args[0].strip() in ("", "void") else len(args)
        out.setdefault(m.group(1), set()).add(n)
    return out


DECL = {k: v for k, v in _calls(_strip_comments(HDR)).items() if not k.endswith("_t")}


@pytest.mark.parametrize("path", ["integration/oai4g_shim.c", "tools/dlsim_tx.c", "tools/dlsim_rx.c"])
def test_callers_match_header(path):
    calls = _calls(_strip_comments(open(os.path.join(ROOT, path)).read()))
    assert calls
    for name, nargs in calls.items():
        assert name in DECL, f"oai4g_{name} not declared in include/oai4g.h"
        assert nargs <= DECL[name], (name, nargs, DECL[name])


def test_shim_entry_points_exported():
    calls = _calls(_strip_comments(open(os.path.join(ROOT, "integration", "oai4g_shim.c")).read()))
    lib = os.path.join(ROOT, "openair4g_amd", "lib", "libopenair4g_amd.so")
    syms = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (oai4g_\w+)", syms))
    for name in calls:
        assert "oai4g_" + name in exported, name


@pytest.mark.parametrize("name", ["dlsim_tx", "dlsim_rx"])
def test_c_drivers_compile_warning_free(tmp_path, name):
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                    "-I", os.path.join(ROOT, "include"), "-c", os.path.join(ROOT, "tools", name + ".c"),
                    "-o", str(tmp_path / "d.o")], check=True)
