"""Static check of inline-asm LDS reads (k_stage1_q8m, k_stage2_*): in the kernel's assembly,
no VALU instruction may read a ds_read destination register before the next s_waitcnt
lgkmcnt (a compiler-inserted copy there reads a register the LDS has not yet written).
Linear scan, conservative about control flow.  python3 scripts/asm_lds_check.py FILE.s SYMBOL"""
import re
import sys


def regs(tok):
    out = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]", tok):
        out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", tok):
        out.add(int(m.group(1)))
    return out


def check(path, sym):
    s = open(path).read()
    a = s.index(sym + ":")
    b = s.index(".Lfunc_end", a)
    pending, bad = set(), []
    for ln in s[a:b].split("\n"):
        t = ln.strip()
        if not t or t.startswith(";"):
            continue
        if t.startswith(("ds_read_b64", "ds_read2_b32", "ds_read_b32", "ds_read2_b64", "ds_read_b128")):
            pending |= regs(t.split()[1].rstrip(","))
            continue
        if t.startswith("s_waitcnt") and "lgkmcnt" in t:
            pending = set()
            continue
        if pending and t.startswith("v_"):
            parts = t.split(None, 1)
            if len(parts) > 1:
                src = set()
                for o in parts[1].split(",")[1:]:
                    src |= regs(o)
                if src & pending:
                    bad.append(t)
    return bad


if __name__ == "__main__":
    bad = check(sys.argv[1], sys.argv[2])
    for t in bad[:10]:
        print("use before wait:", t)
    print("%d suspicious instructions" % len(bad))
    sys.exit(1 if bad else 0)
