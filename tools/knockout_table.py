"""Per-class instruction and cycle attribution of the wheel kernel from
knockout builds (tools/instrument_knockout.py, tools/gpu/knockout_pmc.sh):
class X's counts = full build (mask 0) - build with X switched off. The
instruction counts are exact; the cycle deltas are an attribution (the
classes overlap in the LDS pipe). Per-mark figures divide by the class's
ds_or instructions (its SQ_INSTS_LDS delta).

  python tools/knockout_table.py gpurun_out/ko 0 1 2 4 8 16 32 15 63
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

NAMES = {1: "A", 2: "B1", 4: "B2", 8: "L", 16: "expand", 32: "init", 15: "all marks", 63: "all"}
KEYS = ["SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_LDS_BANK_CONFLICT",
        "SQ_LDS_IDX_ACTIVE", "cyc"]


def main():
    root, masks = sys.argv[1], [int(m) for m in sys.argv[2:]]
    v = {}
    for m in masks:
        d = load(os.path.join(root, f"ko{m}"), "wheel_segments_kernel")
        d["cyc"] = d.get("GRBM_GUI_ACTIVE", 0) / 8  # cycles per CU (8 XCDs)
        v[m] = d
    base = v[0]
    print(f"full build: kernel {base['cyc'] / 2.4e6:.3f} ms at 2.4 GHz; " +
          ", ".join(f"{k} {base[k]:.3e}" for k in KEYS[:-1]))
    print(f"{'class':10s} {'ds_or':>10s} {'VALU':>10s} {'SALU':>10s} {'branch':>10s} {'bank-cfl':>10s} "
          f"{'LDS-busy':>10s} {'ms':>7s} | {'VALU/ds':>7s} {'SALU/ds':>7s} {'cfl/ds':>7s} {'CUcyc/ds':>8s}")
    for m in masks:
        if m == 0:
            continue
        d = {k: base[k] - v[m][k] for k in KEYS}
        n = d["SQ_INSTS_LDS"]
        per = lambda k: d[k] / n if n > 0 else float("nan")  # noqa: E731
        cu_cyc = d["cyc"] * 256 / n if n > 0 else float("nan")  # CU-cycles per wave-level ds_or
        print(f"{NAMES.get(m, m):10s} {n:10.3e} {d['SQ_INSTS_VALU']:10.3e} {d['SQ_INSTS_SALU']:10.3e} "
              f"{d['SQ_INSTS_BRANCH']:10.3e} {d['SQ_LDS_BANK_CONFLICT']:10.3e} {d['SQ_LDS_IDX_ACTIVE']:10.3e} "
              f"{d['cyc'] / 2.4e6:7.3f} | {per('SQ_INSTS_VALU'):7.2f} {per('SQ_INSTS_SALU'):7.2f} "
              f"{per('SQ_LDS_BANK_CONFLICT'):7.2f} {cu_cyc:8.2f}")


if __name__ == "__main__":
    main()
