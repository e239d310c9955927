"""Per-shape table of the hand-written projection GEMMs (csrc/stream_gemm.hip) from a rocprofv3 kernel_stats.csv of
the C2 step: average time per launch, algorithmic HBM bytes and FLOPs per launch, achieved GB/s and TF/s.

    python tools/sgemm_table.py <run_kernel_stats.csv> [M]

M = rows of one attention block (C2: 32 snapshots x 10,000 nodes = 320,000; the temporal block has the same count).
Bytes are algorithmic: every operand read once, every output written once (fp32 = 4 B, bf16 = 2 B per element; the
LN prologue reads x and writes 8 B of statistics per row; the LN-recomputing weight gradient reads x fp32 and 8 B of
statistics per row; the LN2 epilogue reads the residual and writes s and y).  TF/s counts the product's own
2·M·N·K FLOPs (fp32-equivalent): in fp32 mode each of those runs as six bf16 plane products on the matrix cores, so the
matrix-core work is 6x that (column `mfma_frac` = 6 (or 1) x TF/s over the 2.5 PF dense bf16 peak).
"""
import csv
import re
import sys

BF16_PEAK_TFS = 2500.0
HBM_PEAK_GBS = 8000.0


def parse(name):
    m = re.search(r"k_sgemm_nt<(\d+), (\d+), (\d+), (\d+), (\d+), (true|false), (true|false), (\d+)(?:, (\d+))?>", name)
    if m:
        K, nsub, nw, _bm, P = (int(m.group(i)) for i in range(1, 6))
        return {"kind": "nt", "K": K, "P": P, "abf": m.group(6) == "true", "cbf": m.group(7) == "true",
                "mode": int(m.group(8)), "nsub": nsub, "nw": nw}
    # ping-pong form (round 6): k_sgemm_nt_pp<K, NSUB, BM, P, ABF, CBF, MODE>, 8 waves
    m = re.search(r"k_sgemm_nt_pp<(\d+), (\d+), (\d+), (\d+), (true|false), (true|false), (\d+)>", name)
    if m:
        return {"kind": "nt", "K": int(m.group(1)), "P": int(m.group(4)), "abf": m.group(5) == "true",
                "cbf": m.group(6) == "true", "mode": int(m.group(7)), "nsub": int(m.group(2)), "nw": 8}
    m = re.search(r"k_sgemm_tn<(\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (true|false), (\d+), (true|false)>", name)
    if m:
        return {"kind": "tn", "N": int(m.group(1)), "K": int(m.group(2)), "P": int(m.group(6)),
                "abf": m.group(7) == "true", "lnx": m.group(9) == "true"}
    return None


def main():
    path = sys.argv[1]
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 320000
    rows = list(csv.DictReader(open(path)))
    out = []
    for r in rows:
        d = parse(r["Name"])
        if d is None:
            continue
        calls = int(r["Calls"])
        avg_us = float(r["TotalDurationNs"]) / calls / 1e3
        if d["kind"] == "nt":
            nsub, nw = d["nsub"], d["nw"]
            N = 16 * nsub * nw
            K = d["K"]
            ea = 2 if d["abf"] else 4
            ec = 2 if d["cbf"] else 4
            mode = d["mode"]
            if mode == 1:
                what, by = "QKV fwd + LN1 prologue", M * (4 * K + N * ec + 8)
            elif mode == 2:
                what, by = "out-proj + LN2 epilogue", M * (K * ea + 4 * N * 3 + 8)
            elif mode == 3:
                what, by = "QKV dX + LN1 bwd epilogue", M * (K * ea + 4 * N * 3 + 8)
            else:
                what = {(128, 384): "QKV fwd", (128, 128): "out-proj fwd / dC", (384, 128): "QKV dX"}.get((K, N), "nt")
                by = M * (K * ea + N * ec)
            fl = 2.0 * M * N * K
            shape = "NT M=%d N=%d K=%d" % (M, N, K)
        else:
            N, K = d["N"], d["K"]
            ea = 2 if d["abf"] else 4
            ex = 4 if d["lnx"] else ea
            by = M * (N * ea + K * ex + (8 if d["lnx"] else 0)) + 4 * (N * K + N)
            fl = 2.0 * M * N * K
            what = ("dW_qkv over LN1(x) recomputed" if d["lnx"] else
                    {384: "dW_qkv", 128: "dW_out"}.get(N, "tn"))
            shape = "TN M=%d N=%d K=%d" % (M, N, K)
        gbs = by / (avg_us * 1e-6) / 1e9
        tfs = fl / (avg_us * 1e-6) / 1e12
        planes_mul = 6 if d["P"] == 3 else 1
        out.append((what, shape, d["P"], calls, avg_us, by / 1e6, gbs, gbs / HBM_PEAK_GBS, tfs,
                    planes_mul * tfs / BF16_PEAK_TFS))
    print("| product | shape | planes | launches | avg us | MB / launch | GB/s | HBM frac | TF/s (fp32-eq) | "
          "mfma_frac |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for o in sorted(out, key=lambda x: -x[3] * x[4]):
        print("| %s | %s | %d | %d | %.1f | %.0f | %.0f | %.2f | %.1f | %.2f |" % o)


if __name__ == "__main__":
    main()
