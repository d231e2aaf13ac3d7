"""Machine check of "compiled unmodified, no stand-in" for every reference library under oracle/_ref
(built by oracle/Makefile from /root/reference):

  - each library's undefined dynamic symbols are libc / libm, the sibling _ref libraries' own
    (reference) definitions, or one of the two logging hooks no test path reaches (logRecord,
    display_backtrace: LOG_x / DevAssert on error branches; the libraries are opened RTLD_LAZY);
  - every symbol our glue files define is on the list below with the reference line it restates or
    stores, so a glue definition cannot quietly take the place of a reference function;
  - no reference TU called a function it had not declared, apart from the names oracle/Makefile's
    ALLOW_* lists carry (each defined later in the same TU, by a sibling reference library, or
    restated in glue as listed): check_implicit.sh fails the build otherwise, and this test re-reads the
    compiler diagnostics it kept (_ref/*.diag)."""
import glob
import os
import re
import subprocess

import pytest

import oracle_lib as O

REF = os.path.join(O.ORACLE_DIR, "_ref")
LIBS = sorted(glob.glob(os.path.join(REF, "libref_*.so")))
pytestmark = pytest.mark.skipif(not os.path.exists("/root/reference") or len(LIBS) < 12,
                                reason="oracle/_ref is verified where the reference tree builds it")

LOG_HOOKS = {"logRecord", "display_backtrace"}
# glue definitions (ours) -> what they are
GLUE = {
    "ref_glue_gold.c": {"ref_glue_lte_gold": "ctypes caller of lte_gold (lte_gold.c:52)"},
    "ref_glue_ofdm.c": {"is_pmch_subframe": "restates pmch.c is_pmch_subframe for num_MBSFN_config = 0",
                        "ref_glue_normal_prefix_mod": "ctypes caller", "ref_glue_do_OFDM_mod": "ctypes caller"},
    "ref_glue_mod.c": {"get_Qm": "restates lte_mcs.c:45-55"},
    "ref_glue_td.c": {"threegpplte_interleaver_output": "storage, lte_interleaver_inline.h:29 (3gpplte.c:42)",
                      "threegpplte_interleaver_tmp": "storage, lte_interleaver_inline.h:30 (3gpplte.c:43)"},
}
ALLOW_IMPLICIT = {"ofdm_mod": {"PHY_ofdm_mod", "is_pmch_subframe"}, "dlsch_modulation": {"get_Qm"},
                  "dlsch_scrambling": {"lte_gold_generic"}, "pcfich": {"lte_gold_generic"},
                  "dlsch_llr_computation": {"qpsk_qpsk", "qpsk_qam16", "qpsk_qam64"}}


def _syms(path, flag):
    out = subprocess.run(["nm", "-D", flag, path], check=True, capture_output=True, text=True).stdout
    return {ln.split()[-1].split("@")[0] for ln in out.splitlines() if ln.strip()}


def _libc_like(name):
    return name.startswith("_") or name in {
        "printf", "puts", "putchar", "fprintf", "fopen", "fclose", "fwrite", "fread", "fflush", "malloc", "calloc",
        "free", "memset", "memcpy", "memmove", "memcmp", "strlen", "strcmp", "strcpy", "strncpy", "sprintf",
        "snprintf", "exit", "abort", "posix_memalign", "sqrt", "log10", "pow", "cos", "sin", "atan2", "atan",
        "floor", "ceil", "fabs", "exp", "log", "sleep", "usleep", "clock_gettime", "gettimeofday", "time",
        "rand", "srand", "random", "srandom", "lrand48", "drand48", "srand48_r", "mrand48_r", "srand48",
        "mrand48", "lround", "round", "sqrtf", "cosf", "sinf", "stderr", "stdout", "perror", "getpid",
        "pthread_mutex_lock", "pthread_mutex_unlock", "backtrace", "backtrace_symbols", "fputs", "fputc",
        "strerror", "memalign", "aligned_alloc", "realloc", "qsort", "atoi", "strtol", "abs", "labs", "vfprintf",
        "vprintf", "fseek", "ftell", "sscanf", "fscanf", "fgets"}


def test_undefined_symbols_are_reference_libc_or_log_hooks():
    defined = {}
    for lib in LIBS:
        for s in _syms(lib, "--defined-only"):
            defined.setdefault(s, os.path.basename(lib))
    for lib in LIBS:
        for s in _syms(lib, "--undefined-only"):
            if _libc_like(s) or s in LOG_HOOKS:
                continue
            owner = defined.get(s)
            assert owner is not None and owner != os.path.basename(lib), (os.path.basename(lib), s)
            assert not any(s in g for g in GLUE.values()) or s == "lte_gold_generic", (os.path.basename(lib), s)


def test_glue_defines_only_the_listed_symbols():
    for src, allowed in GLUE.items():
        obj = os.path.join(REF, src.replace(".c", ".o"))
        out = subprocess.run(["nm", "--defined-only", obj], check=True, capture_output=True, text=True).stdout
        text_syms = {ln.split()[-1] for ln in out.splitlines() if ln.split()[1] in "TDBC"}
        extra = {s for s in text_syms - set(allowed) if not s.startswith("ref_glue_")}
        if src == "ref_glue_mod.c":    # table storage from the reference's own PHY/LTE_TRANSPORT/vars.h and
            hdrs = "".join(open(h).read() for h in    # the table headers it includes, all unmodified
                           glob.glob("/root/reference/openair1/PHY/LTE_TRANSPORT/*.h"))
            extra = {s for s in extra if not re.search(r"\b%s\b" % re.escape(s), hdrs)}
        assert not extra, (src, sorted(extra))


def test_implicit_declarations_are_only_the_allowlisted():
    diags = glob.glob(os.path.join(REF, "*.diag"))
    assert len(diags) >= 20
    for dg in diags:
        tu = os.path.basename(dg)[:-5]
        names = set(re.findall(r"implicit declaration of function '([^']+)'", open(dg).read()))
        assert names <= ALLOW_IMPLICIT.get(tu, set()), (tu, names)
    mk = open(os.path.join(O.ORACLE_DIR, "Makefile")).read()
    for tu, names in ALLOW_IMPLICIT.items():
        m = re.search(r"^ALLOW_%s = (.*)$" % tu, mk, re.M)
        assert m and set(m.group(1).split()) == names, tu
