"""gfx950 ISA audit of the built HIP library (run by csrc/Makefile after every link and by tests/test_isa_audit.py).

Finding (round 6, DESIGN.md section 5 "The round-5 dgamma glitch"): on MI355X under ROCm 7.2 a packed-FP32 VALU
instruction whose op_sel feeds the LOW lane from src1's HIGH register (e.g. ``v_pk_mul_f32 v[96:97], v[94:95],
v[180:181] op_sel:[0,1] op_sel_hi:[1,0]``) intermittently yields a dropped (zero) low-lane product for one 16-lane
quarter of the wave; the same product with the select on src0 is exact (profiles/r6d_ln2_isa_bisect.txt).  The
compiler's hazard recognizer does not know it, so the library must not contain the form.  This audit disassembles
every gfx950 code object in the shared library and lists each ``v_pk_{add,mul,fma}_f32`` whose op_sel has a 1 for
src1 or src2.  Exit status 1 when any is found.

    python tools/isa_audit.py <lib.so> [--all]    (--all: also print the per-form census of packed-FP32 selects)
"""
import collections
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
PK = re.compile(r"\bv_pk_(add|mul|fma)_f32\b(.*)$")
OPSEL = re.compile(r"\bop_sel:\[([01,]+)\]")


def fatbin(path):
    """The .hip_fatbin section's bytes (ELF64 little-endian section headers, no external tools)."""
    d = open(path, "rb").read()
    shoff, = struct.unpack_from("<Q", d, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", d, 0x3A)
    sh = [struct.unpack_from("<IIQQQQIIQQ", d, shoff + i * shentsize) for i in range(shnum)]
    stro = sh[shstrndx][4]
    for name, _t, _f, _a, off, size, *_ in sh:
        n = d[stro + name: d.index(b"\0", stro + name)]
        if n == b".hip_fatbin":
            return d[off: off + size]
    raise SystemExit(f"{path}: no .hip_fatbin section")


def code_objects(path, arch="gfx950"):
    """Every ``arch`` code object of every clang offload bundle in the library."""
    fb = fatbin(path)
    out = []
    pos = fb.find(MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fb, pos + len(MAGIC))
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fb, p)
            triple = fb[p + 24: p + 24 + tlen].decode()
            p += 24 + tlen
            if arch in triple and size:
                out.append(fb[pos + off: pos + off + size])
        pos = fb.find(MAGIC, pos + 1)
    return out


def disassemble(co):
    with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
        f.write(co)
        name = f.name
    try:
        return subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", name], text=True)
    finally:
        os.remove(name)


def forbidden(ins: str) -> bool:
    """A packed-FP32 instruction whose op_sel selects src1's (or src2's) high register for the low lane."""
    m = PK.search(ins)
    if not m:
        return False
    sel = OPSEL.search(m.group(0))
    return bool(sel) and any(int(b) for b in sel.group(1).split(",")[1:])


def audit(path):
    """(findings, census): findings = [(kernel, instruction)] of the forbidden form; census = Counter of op_sel forms."""
    findings, census = [], collections.Counter()
    cos = code_objects(path)
    if not cos:
        raise SystemExit(f"{path}: no gfx950 code object")
    for co in cos:
        fn = "?"
        for line in disassemble(co).splitlines():
            if line.endswith(">:"):
                fn = line.split("<", 1)[1][:-2]
                continue
            m = PK.search(line)
            if not m:
                continue
            ins = m.group(0).split("//")[0].strip()
            census[ins.split(" ", 1)[0] + " " + " ".join(t for t in ins.split() if t.startswith(("op_sel", "neg")))] += 1
            if forbidden(ins):
                findings.append((fn, ins))
    return findings, census


def main(argv):
    if not argv:
        print(__doc__)
        return 2
    findings, census = audit(argv[0])
    if "--all" in argv:
        for k, v in census.most_common():
            print(f"{v:7d}  {k}")
    for fn, ins in findings:
        print(f"FORBIDDEN packed-FP32 src1/src2 high select in {fn}: {ins}")
    print(f"isa_audit {os.path.basename(argv[0])}: {sum(census.values())} packed-FP32 instructions, "
          f"{len(findings)} with a src1/src2 high select")
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
