"""Instruction mix per region of a kernel's assembly listing (profiling aid).

Build the listing with the region comments of the phase markers:
  hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -Iinclude -Icrypto-recommendation_amd/csrc \
        -DLSHKM_ISA_MARK -x hip -S --cuda-device-only crypto-recommendation_amd/csrc/fused.hip -o /tmp/fused.s
then: python tools/isa_regions.py /tmp/fused.s 'fused_hi_kernelILb1ELb0ELi0ELi1ELb1ELi0E'
Regions are the text between consecutive ';PTMARK i' comments (static counts:
unrolled loops count every copy, loops with a runtime trip count once).
"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_cmp", "v_cndmask")):
        return "valu_cmp"
    if op.startswith(("v_add_f64", "v_mul_f64", "v_fma_f64", "v_cvt_f64", "v_cvt_f32_f64", "v_sqrt_f64", "v_div", "v_ldexp_f64",
                      "v_frexp", "v_rcp_f64", "v_rsq_f64")):
        return "valu_f64"
    if op.startswith(("v_accvgpr", "v_mov", "v_permlane")):
        return "valu_move"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main(path, sym):
    text = open(path).read().splitlines()
    start = next(i for i, l in enumerate(text) if l.startswith("_ZN") and sym in l.split(":")[0] and ":" in l)
    end = next(i for i in range(start + 1, len(text)) if text[i].strip().startswith(".Lfunc_end"))
    regions, cur, name = [], Counter(), "start"
    for l in text[start:end]:
        s = l.strip()
        m = re.match(r";PTMARK (\d+)", s)
        if m:
            regions.append((name, cur))
            cur, name = Counter(), f"after mark {m.group(1)}"
            continue
        if not s or s.startswith((";", ".", "_")) or s.split(";")[0].rstrip().endswith(":"):
            continue
        cur[classify(s.split()[0])] += 1
    regions.append((name, cur))
    keys = ["mfma", "valu", "valu_f64", "valu_cmp", "valu_move", "lds", "vmem", "salu", "wait"]
    print(f"{'region':16s} " + " ".join(f"{k:>9s}" for k in keys))
    for n, c in regions:
        print(f"{n:16s} " + " ".join(f"{c[k]:9d}" for k in keys))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
