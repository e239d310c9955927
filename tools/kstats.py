"""Summarise a rocprofv3 kernel_stats.csv per training step, grouped by kernel family.

    python tools/kstats.py <run_kernel_stats.csv> [steps]

steps defaults to the number of k_geo_fwd launches / 2 (two geometric layers per step).
"""
import csv
import re
import sys

FAMILIES = [
    ("sgemm (hand-written)", r"k_sgemm|k_rowgemm"),
    ("gemm", r"^Cijk_|gemm|Gemm"),
    ("geo", r"k_geo_"),
    ("temporal", r"k_tattn"),
    ("layernorm", r"k_ln_"),
    ("LN2 bwd + out-proj grads (fused)", r"k_ln2_bwd_out"),
    ("proj (fused MFMA)", r"k_proj"),
    ("csr", r"rocprim|k_scatter|k_fill_tail|k_keys|k_chunk|k_tri|csr|csc|k_count|k_part_|k_refine|k_big_list|k_init\(|scan::k_|Tri"),
    ("colsum/pool", r"k_colsum|k_pool"),
    ("embedding (narrow)", r"k_narrow"),
    ("head / bias table / params", r"k_head_|k_bias_table|k_qkv_|k_sgemm_wprep"),
    ("torch elementwise", r"elementwise|CatArray|index|gather|scatter"),
    ("torch reduce", r"reduce_kernel"),
    ("fill/copy", r"__amd_rocclr"),
]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n_geo = sum(int(r["Calls"]) for r in rows if "k_geo_fwd_chunk" in r["Name"])
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else max(1, n_geo / 2)
    tot = {}
    top = []
    for r in rows:
        fam = next((f for f, p in FAMILIES if re.search(p, r["Name"])), "other")
        ns = float(r["TotalDurationNs"])
        tot[fam] = tot.get(fam, 0.0) + ns
        top.append((ns, int(r["Calls"]), r["Name"][:110]))
    all_ms = sum(tot.values()) / steps / 1e6
    print("steps=%g  device ms/step=%.3f" % (steps, all_ms))
    for f, ns in sorted(tot.items(), key=lambda x: -x[1]):
        print("  %-18s %7.3f ms" % (f, ns / steps / 1e6))
    print("top kernels (ms/step, calls/step):")
    for ns, c, n in sorted(top, reverse=True)[:25]:
        print("  %7.3f %5.1f  %s" % (ns / steps / 1e6, c / steps, n))


if __name__ == "__main__":
    main()
