"""Instruction mix of a kernel's hottest loop in a hipcc -S listing (test / measurement infrastructure).

The hottest loop is taken as the largest basic-block range closed by a backward branch (s_cbranch_* to an
earlier label).  Prints the instruction classes in it; with --per N, per N units of work (e.g. the element-
restart pairs one trip of an unrolled loop processes).  Usage:
    python tools/isa_loop.py <file.s> <kernel-name-substring> [--per N]
"""
import collections
import re
import sys


def kernel_body(lines, sub):
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*" + re.escape(sub) + r"\S*:", l):
            start = i
        elif start is not None and "s_endpgm" in l:
            return lines[start:i + 1]
    raise SystemExit(f"kernel {sub!r} not found")


def hottest_loop(body):
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    best = None
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)", l) or re.search(r"s_branch\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            seg = body[labels[m.group(1)]:i + 1]
            n = sum(1 for x in seg if re.match(r"^\s+[sv]_|^\s+ds_|^\s+buffer_|^\s+global_", x))
            if best is None or n > best[0]:
                best = (n, seg)
    return best[1] if best else []


def innermost_loop_with(body, opcode):
    """The instructions of the smallest backward-branch loop of `body` that contains `opcode` (e.g. the unrolled
    inner loop of a kernel, without the tile loop around it)."""
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    best = None
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)", l) or re.search(r"s_branch\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            seg = [x.strip() for x in body[labels[m.group(1)]:i + 1]
                   if re.match(r"^\s+[a-z_]+[0-9a-z_]*\s", x) and not x.strip().startswith((";", "."))]
            if any(x.split()[0].startswith(opcode) for x in seg) and (best is None or len(seg) < len(best)):
                best = seg
    return best or []


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_fma_f64", "v_fmac_f64")):
        return "v_fma_f64"
    if op.startswith("v_rcp_f64"):
        return "v_rcp_f64"
    if op.startswith("v_") and "f64" in op:
        return "valu_f64_other"
    if op.startswith("v_"):
        return "valu_32bit"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_store"
    if op.startswith("s_waitcnt") or op.startswith("s_barrier") or op.startswith("s_nop"):
        return "wait/barrier/nop"
    if op.startswith("s_"):
        return "salu/branch"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    per = int(sys.argv[sys.argv.index("--per") + 1]) if "--per" in sys.argv else 1
    lines = open(path).read().splitlines()
    loop = hottest_loop(kernel_body(lines, sub))
    ins = [x.strip() for x in loop if re.match(r"^\s+[a-z_]+[0-9a-z_]*\s", x) and not x.strip().startswith(";")]
    ins = [x for x in ins if not x.startswith(".")]
    c = collections.Counter(classify(x) for x in ins)
    print(f"{sub}: hottest loop {len(ins)} instructions" + (f", per unit (/{per}):" if per > 1 else ":"))
    for k, v in sorted(c.items(), key=lambda kv: -kv[1]):
        print(f"  {k:18s} {v:6d}" + (f"  {v / per:8.2f}" if per > 1 else ""))


if __name__ == "__main__":
    main()
