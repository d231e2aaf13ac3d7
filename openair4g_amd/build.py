"""Build the in-tree HIP shared library (gfx950) and the CPU oracle.

The product library is compiled with hipcc straight into openair4g_amd/lib/ so that it
travels with the repository snapshot to the GPU box.  No JIT, no cache outside the tree.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libopenair4g_amd.so")
SOURCES = ["oai4g_host.cpp", "oai4g_encode.hip", "oai4g_ofdm.hip", "oai4g_decode.hip", "oai4g_decode8.hip", "oai4g_fep.hip", "oai4g_ctrl.hip", "oai4g_rx.hip", "oai4g_chest.hip", "oai4g_channel.hip", "oai4g_dist.cpp"]
EXTRA = [os.path.join(ROOT, "include", "oai4g_qpp.c"), os.path.join(ROOT, "include", "oai4g_tbs.c")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("OAI4G_ARCH", "gfx950")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force=False, verbose=False, out=None, defines=(), only=None):
    """Compile the library; `out`/`defines` build a variant (e.g. -DOAI4G_MODOFDM_WAVES=3); with
    `only` (source basenames) a variant recompiles just those and links the in-tree objects of
    the others."""
    lib = out or LIB
    libdir = os.path.dirname(lib)
    os.makedirs(libdir, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + EXTRA + [os.path.join(CSRC, "oai4g_internal.h"), os.path.join(CSRC, "oai4g_dft_prims.h"), os.path.join(ROOT, "include", "oai4g.h")]
    if not force and not _newer(lib, deps):
        return lib
    objs = []
    hdrs = deps[len(srcs) + len(EXTRA):] + [os.path.join(ROOT, "include", "oai4g_qpp.h"),
                                             os.path.join(ROOT, "include", "oai4g_tbs.h")]
    for src in srcs + EXTRA:
        obj = os.path.join(libdir, os.path.basename(src) + ".o")
        if only is not None and os.path.basename(src) not in only:
            objs.append(os.path.join(LIBDIR, os.path.basename(src) + ".o"))
            continue
        if not force and not defines and not _newer(obj, [src] + hdrs):   # incremental: unchanged objects stay
            objs.append(obj)
            continue
        lang = ["-x", "hip"] if src.endswith((".hip", ".cpp")) else ["-x", "c"]
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-Wall", "-Wno-unused-result", "-Wno-unused-value",
               "-I", os.path.join(ROOT, "include")] + list(defines) + (["-std=c++17"] if lang[1] == "hip" else []) + lang + \
              ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        objs.append(obj)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs + ["-L/opt/rocm/lib", "-lrccl", "-lpthread",
                                                                                "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return lib


def build_host_tools(verbose=False):
    """gcc-built C host programs over the C ABI: tools/dlsim_tx.c (dlsim's transmit loop) and
    tools/dlsim_rx.c (the whole downlink loop, eNB to decoded transport blocks) -> tools/bin/."""
    outs = []
    for name in ("dlsim_tx", "dlsim_rx"):
        out = os.path.join(ROOT, "tools", "bin", name)
        src = os.path.join(ROOT, "tools", name + ".c")
        outs.append(out)
        if not _newer(out, [src, LIB, os.path.join(ROOT, "include", "oai4g.h")]):
            continue
        os.makedirs(os.path.dirname(out), exist_ok=True)
        cmd = ["gcc", "-O2", "-std=gnu11", "-Wall", "-I", os.path.join(ROOT, "include"), src, "-L", LIBDIR,
               "-lopenair4g_amd", "-Wl,-rpath,$ORIGIN/../../openair4g_amd/lib", "-o", out]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return outs[0]


def build_oracle(verbose=False):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)


def build_shim(verbose=False):
    """integration/liboai4g_shim.so: the reference-side boundary compiled against the reference's own
    headers (only where /root/reference exists; the built .so travels with the tree)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "integration")], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)


if __name__ == "__main__":
    if "--variant" in sys.argv:   # build.py --variant NAME -DFOO=1 [-mllvm X] ... -> variants/NAME/libopenair4g_amd.so
        i = sys.argv.index("--variant")
        rest = [a for a in sys.argv[i + 2:] if a != "--force"]
        only = [a[len("--only="):] for a in rest if a.startswith("--only=")] or None
        name, defs = sys.argv[i + 1], [a for a in rest if not a.startswith("--only=")]
        print("built", build_lib(force=True, out=os.path.join(ROOT, "variants", name, "libopenair4g_amd.so"),
                                 defines=defs, only=only))
        sys.exit(0)
    build_lib(force="--force" in sys.argv, verbose=True)
    build_host_tools(verbose=True)
    build_oracle(verbose=True)
    build_shim(verbose=True)
    print("built", LIB)
