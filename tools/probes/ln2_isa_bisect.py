"""GPU side of the round-6 k_ln2_bwd_out ISA bisection (tools/probes/ln2_isa_variants.py builds the code objects).

Launches k_ln2_bwd_out<1, fp32, skip> from each code object with hipModuleLaunchKernel (same L2Args, grid and LDS as
tagan_ln2_bwd_out), three calls per case, and reports: bitwise reproducibility of the per-workgroup LN partials,
dgamma against fp64, and for every wrong (workgroup, column) partial the single-row explanation that fits its error
best (row dropped / doubled / paired with the same thread's next- or previous-tile operand).
"""
import ctypes
import glob
import os
import struct
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import tagan_amd  # noqa: E402
from tagan_amd import stream_gemm as sg  # noqa: E402

KERNEL = b"_ZN5tagan12_GLOBAL__N_113k_ln2_bwd_outILi1ELb0ELb1EEEvNS0_6L2ArgsE"
H, BM = 128, 32
dev = torch.device("cuda:0")
torch.zeros(1, device=dev)
hip = ctypes.CDLL([l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l][0])
hip.hipModuleLaunchKernel.argtypes = [ctypes.c_void_p] + [ctypes.c_uint] * 7 + [ctypes.c_void_p] * 3


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: hip error {rc}")


def load(path):
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    check(hip.hipModuleLoad(ctypes.byref(mod), path.encode()), "hipModuleLoad " + path)
    check(hip.hipModuleGetFunction(ctypes.byref(fn), mod, KERNEL), "hipModuleGetFunction")
    return fn


def ln64(x, eps=1e-5):
    x = x.double()
    m = x.mean(1, keepdim=True)
    v = ((x - m) ** 2).mean(1, keepdim=True)
    return m[:, 0], (1.0 / torch.sqrt(v + eps))[:, 0]


def case(M):
    g = torch.Generator(device=dev).manual_seed(M)
    s = 0.2 + torch.randn(M, H, device=dev, generator=g)
    dy = torch.randn(M, H, device=dev, generator=g)
    c = torch.randn(M, H, device=dev, generator=g)
    w = torch.randn(H, H, device=dev, generator=g) / H ** 0.5
    xs = torch.randn(M, H, device=dev, generator=g)
    gs = 1 + 0.1 * torch.randn(H, device=dev, generator=g)
    lw = 1 + 0.1 * torch.randn(H, device=dev, generator=g)
    m, r = ln64(s)
    ms, rs = ln64(xs)
    return dict(M=M, s=s, dy=dy, c=c, wp=sg.wprep(w, True, 1), xs=xs, gs=gs, lw=lw, m=m.float(), r=r.float(),
                ms=ms.float(), rs=rs.float(), xh=(s.double() - m[:, None]) * r[:, None])


def launch(fn, k):
    M = k["M"]
    tiles = (M + BM - 1) // BM
    G = min(tiles, 256)
    tpw = (tiles + G - 1) // G
    dres = torch.empty(M, H, device=dev)
    dc = torch.empty(M, H, device=dev)
    part_w = torch.empty(G, H * H + H, device=dev)
    part_ln = torch.empty(G, 4 * H, device=dev)
    p = lambda t: t.data_ptr()
    args = struct.pack("<qqQQQQQffQQQQQQQQQQQQ", M, tpw, p(k["dy"]), p(k["s"]), p(k["m"]), p(k["r"]), p(k["lw"]),
                       0.0, 1.0, 0, 0, p(k["xs"]), p(k["ms"]), p(k["rs"]), p(k["gs"]), p(k["c"]), p(k["wp"]),
                       p(dres), p(dc), p(part_w), p(part_ln))
    assert len(args) == 160
    buf = ctypes.create_string_buffer(args, len(args))
    size = ctypes.c_size_t(len(args))
    extra = (ctypes.c_void_p * 5)(1, ctypes.cast(buf, ctypes.c_void_p), 2, ctypes.cast(ctypes.byref(size),
                                                                                       ctypes.c_void_p), 3)
    lds = 2 * 1 * BM * (H + 16) * 2 + 8 * 4 * H * 4
    check(hip.hipModuleLaunchKernel(fn, G, 1, 1, 512, 1, 1, lds, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
                                    None, extra), "launch")
    torch.cuda.synchronize()
    return part_ln.view(G, 4, H).clone(), tpw


def explain(k, part, tpw, limit=int(os.environ.get("EXPLAIN", "6"))):
    """Per-workgroup dgamma partials vs fp64; the best single-row explanation of each wrong one."""
    M, dy, xh = k["M"], k["dy"].double(), k["xh"]
    cr = dy * xh
    out = []
    G = part.shape[0]
    for b in range(G):
        r0, r1 = b * tpw * BM, min((b + 1) * tpw * BM, M)
        if r0 >= r1:
            continue
        ref = cr[r0:r1].sum(0)
        scale = cr[r0:r1].abs().sum(0)
        err = part[b, 0].double() - ref
        for col in (err.abs() > 1e-5 * scale).nonzero().flatten().tolist():
            rows = torch.arange(r0, r1, device=dev)
            nxt = torch.clamp(rows + BM, max=M - 1)
            prv = torch.clamp(rows - BM, min=0)
            cands = {"dropped": -cr[rows, col], "doubled": cr[rows, col],
                     "dy_next_tile": dy[nxt, col] * xh[rows, col] - cr[rows, col],
                     "xh_next_tile": dy[rows, col] * xh[nxt, col] - cr[rows, col],
                     "dy_prev_tile": dy[prv, col] * xh[rows, col] - cr[rows, col],
                     "xh_prev_tile": dy[rows, col] * xh[prv, col] - cr[rows, col]}
            best = min(((float((err[col] - v).abs().min()), n, int((err[col] - v).abs().argmin()) + r0)
                        for n, v in cands.items()))
            out.append((b, col, float(err[col]), best))
    for b, col, e, (res, n, row) in out[:limit]:
        print(f"    wg {b} col {col} (8q+{col % 8}) err {e:+.4e}  best: {n} row {row} (tile {(row - b * tpw * BM) // BM}"
              f" of {tpw}, tile row {row % BM}) residual {res:.1e}", flush=True)
    cols = sorted({col for _, col, _, _ in out})
    print(f"    wrong partials: {len(out)} in {len({b for b, _, _, _ in out})} workgroups; columns {cols[:16]}",
          flush=True)


def main():
    paths = sorted(glob.glob(os.path.join(ROOT, "tools", "probes", "ln2_isa", "*.hsaco")))
    cases = [case(M) for M in (40961, 320000)]
    for path in paths:
        fn = load(path)
        for k in cases:
            parts = [launch(fn, k) for _ in range(int(os.environ.get("CALLS", "3")))]
            det = all(torch.equal(parts[0][0], x[0]) for x in parts[1:])
            dg = parts[0][0][:, 0].double().sum(0)
            ref = (k["dy"].double() * k["xh"]).sum(0)
            rel = float((dg - ref).abs().max() / ref.abs().max())
            print(f"{os.path.basename(path)} M={k['M']} deterministic={det} dgamma maxrel={rel:.2e}", flush=True)
            if not det or rel > 1e-5:
                for i, (pl, tpw) in enumerate(parts):
                    print(f"  call {i}:", flush=True)
                    explain(k, pl, tpw)


if __name__ == "__main__":
    main()
