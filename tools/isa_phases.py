"""Static instruction mix of one kernel's persistent item loop, split at its s_barrier boundaries
(diagnostic).  usage: python tools/isa_phases.py <file.s> <mangled kernel name> [seg labels...]

Build the assembly with the library's flags plus --cuda-device-only -S, e.g.
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -x hip --cuda-device-only -S \
        openair4g_amd/csrc/oai4g_ofdm.hip -o /tmp/ofdm.s
Every instruction between two barriers is counted once (the loop body is straight-line code apart
from the cold zero-symbol path, whose lines are listed separately).  VALU classes: dot2 (v_dot2*),
pk (v_pk_*), cvt_pk (v_cvt_pk*), other VALU (v_*), LDS (ds_*), VMEM (global_* / buffer_*), SALU (s_*
except waits / branches / barriers)."""
import re
import sys


def classify(op):
    if op.startswith("v_dot2"):
        return "dot2"
    if op.startswith("v_pk_"):
        return "pk"
    if op.startswith("v_cvt_pk"):
        return "cvt_pk"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith(("s_waitcnt", "s_barrier", "s_branch", "s_cbranch", "s_nop", "s_endpgm", "s_setprio")):
        return "ctl"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    path, name = sys.argv[1], sys.argv[2]
    labels = sys.argv[3:]
    s = open(path).read().split("\n")
    start = next(i for i, l in enumerate(s) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
    body = s[start:end]
    # the item loop: the last "=>This Loop Header" with Depth=1, to its back edge
    head = max(i for i, l in enumerate(body) if "=>This Loop Header" in l and "Depth=1" in l)
    segs, cur = [], []
    for l in body[head:]:
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        if op == "s_barrier":
            segs.append(cur)
            cur = []
            continue
        cur.append(op)
    segs.append(cur)
    cols = ["dot2", "pk", "cvt_pk", "valu", "lds", "vmem", "salu"]
    print(f"{'segment':28s} " + " ".join(f"{c:>7s}" for c in cols) + "   VALU total")
    tot = {c: 0 for c in cols}
    for k, seg in enumerate(segs):
        cnt = {c: 0 for c in cols}
        for op in seg:
            c = classify(op)
            if c in cnt:
                cnt[c] += 1
        v = cnt["dot2"] + cnt["pk"] + cnt["cvt_pk"] + cnt["valu"]
        for c in cols:
            tot[c] += cnt[c]
        lab = labels[k] if k < len(labels) else f"seg {k}"
        print(f"{lab:28s} " + " ".join(f"{cnt[c]:7d}" for c in cols) + f"   {v:6d}")
    v = tot["dot2"] + tot["pk"] + tot["cvt_pk"] + tot["valu"]
    print(f"{'total':28s} " + " ".join(f"{tot[c]:7d}" for c in cols) + f"   {v:6d}")


if __name__ == "__main__":
    main()
