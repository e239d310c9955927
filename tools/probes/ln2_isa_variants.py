"""Round-6 ISA bisection of the round-5 k_ln2_bwd_out nondeterminism (Next 1).

Builds gfx950 code objects of stream_gemm.hip's device code with TAGAN_LN2_FORM=2 (the round-5 first form, which
reproduces the wrong dgamma columns 8q + 4: profiles/r6b_ln2_first_form_probe.txt) and hand-edited variants of its
emitted assembly, each a one-line change in k_ln2_bwd_out<1, fp32, skip>.  tools/probes/ln2_isa_bisect.py runs them
on the GPU through hipModuleLoad.  Run here (no GPU needed):  python tools/probes/ln2_isa_variants.py
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "temporal-asymmetric-graph-attention-network_amd", "csrc")
OUT = os.path.join(ROOT, "tools", "probes", "ln2_isa")
LLVM = "/opt/rocm/lib/llvm/bin"
KERNEL = "_ZN5tagan12_GLOBAL__N_113k_ln2_bwd_outILi1ELb0ELb1EEEvNS0_6L2ArgsE"


def compile_asm(form: int) -> list:
    s = os.path.join(OUT, f"form{form}.s")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                           f"-DTAGAN_LN2_FORM={form}", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
                           "--cuda-device-only", "-S", os.path.join(CSRC, "stream_gemm.hip"), "-o", s],
                          stderr=subprocess.DEVNULL)
    return open(s).read().split("\n")


def kernel_range(lines):
    a = lines.index(KERNEL + ": ; @" + KERNEL)
    b = next(i for i in range(a, len(lines)) if lines[i].strip().startswith(".end_amdhsa_kernel"))
    return a, b


def find(lines, a, b, text, nth=0):
    hits = [i for i in range(a, b) if lines[i].strip() == text]
    if len(hits) <= nth:
        raise SystemExit(f"pattern not found: {text!r} ({len(hits)} hits)")
    return hits[nth]


def variants(lines):
    a, b = kernel_range(lines)
    e4 = "v_pk_mul_f32 v[96:97], v[94:95], v[180:181] op_sel:[0,1] op_sel_hi:[1,0]"
    last_load = "global_load_dword v193, v[100:101], off"        # the loop's last next-tile load
    sums0 = "v_pk_mul_f32 v[100:101], v[96:97], v[186:187]"     # first instruction of the LN column sums
    e6 = "v_pk_mul_f32 v[100:101], v[96:97], v[184:185] op_sel:[0,1] op_sel_hi:[1,0]"
    out = {"v0_asis": list(lines)}
    v = list(lines); v.insert(find(v, a, b, last_load) + 1, "\ts_waitcnt vmcnt(0)"); out["v1_wait_after_loads"] = v
    v = list(lines); v[find(v, a, b, e4)] = "\tv_mul_f32_e32 v96, v94, v181"; out["v2_e4_plain_mul"] = v
    v = list(lines); v.insert(find(v, a, b, e4), "\ts_nop 7"); out["v3_nop_before_e4"] = v
    v = list(lines); v.insert(find(v, a, b, sums0), "\ts_waitcnt vmcnt(0)"); out["v4_wait_before_sums"] = v
    v = list(lines); v.insert(find(v, a, b, e4) + 1, "\ts_nop 7"); out["v5_nop_after_e4"] = v
    if os.environ.get("LN2_ROUND") == "2":   # second bisection round: padding width, commuted operands, MFMA drain
        out = {"v0_asis": list(lines)}
        for n in (0, 1, 3, 7):
            v = list(lines)
            for t in (e4, e6):
                v.insert(find(v, a, b, t), f"\ts_nop {n}")
            out[f"w{n}_nop{n}_before_e4_e6"] = v
        v = list(lines)
        v[find(v, a, b, e4)] = "\tv_pk_mul_f32 v[96:97], v[180:181], v[94:95] op_sel:[1,0] op_sel_hi:[0,1]"
        v[find(v, a, b, e6)] = "\tv_pk_mul_f32 v[100:101], v[184:185], v[96:97] op_sel:[1,0] op_sel_hi:[0,1]"
        out["x_commuted_e4_e6"] = v
        v = list(lines)
        i = find(v, a, b, sums0)
        v[i:i] = ["\ts_nop 7"] * 16
        out["y_mfma_drain_before_sums"] = v
    return out


def assemble(name, lines):
    s = os.path.join(OUT, name + ".s")
    o = os.path.join(OUT, name + ".o")
    h = os.path.join(OUT, name + ".hsaco")
    open(s, "w").write("\n".join(lines))
    subprocess.check_call([f"{LLVM}/clang", "-target", "amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c", s, "-o", o])
    subprocess.check_call([f"{LLVM}/ld.lld", "-shared", o, "-o", h])
    os.remove(o)
    os.remove(s)
    return h


def main():
    os.makedirs(OUT, exist_ok=True)
    for f in os.listdir(OUT):
        os.remove(os.path.join(OUT, f))
    lines = compile_asm(2)
    for name, v in variants(lines).items():
        print(assemble(name, v))
    if os.environ.get("LN2_ROUND") != "2":
        assemble("f0_shipped", compile_asm(0))
    for f in ("form2.s", "form0.s"):
        if os.path.exists(os.path.join(OUT, f)):
            os.remove(os.path.join(OUT, f))


if __name__ == "__main__":
    sys.exit(main())
