"""Per-launch PMC figures of the wheel kernel from tools/gpu/pmc_deep.sh's
CSVs: rows of one dispatch and counter are summed (rocprofv3 may split a
counter over rows), then averaged over dispatches. Derived: cycles per CU
(GRBM_GUI_ACTIVE / 8 XCDs), VALU/LDS/SALU instructions per CU-cycle, wave
state shares (SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY =
SQ_WAVE_CYCLES), average in-flight LDS / VMEM instructions.

  python tools/pmc_summary.py gpurun_out/<dir> [kernel-substring]
"""
import collections
import csv
import glob
import os
import sys

NUM_CUS = 256


def load(root, pat):
    """Dispatches of the largest grid only (a range's tail may be a second,
    half-geometry launch of the same kernel name)."""
    rows = []
    for f in glob.glob(os.path.join(root, "pmc_*.csv")):
        rows += [(os.path.basename(f), r) for r in csv.DictReader(open(f)) if pat in r["Kernel_Name"]]
    if not rows:
        return {}
    grid = max(int(r["Grid_Size"]) for _, r in rows)
    v = collections.defaultdict(lambda: collections.defaultdict(float))
    for f, r in rows:
        if int(r["Grid_Size"]) == grid:
            v[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    return {k: sum(d.values()) / len(d) for k, d in v.items()}


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "wheel_segments_kernel"
    v = load(root, pat)
    for k in sorted(v):
        print(f"{k:28s} {v[k]:.4e}")
    cyc = v.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc:
        print(f"cycles per CU                {cyc:.4e}")
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT"):
            if k in v:
                print(f"{k + ' per CU-cycle':28s} {v[k] / NUM_CUS / cyc:.3f}")
    wc = v.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM"):
            if k in v:
                print(f"{k + ' / WAVE_CYCLES':28s} {v[k] / wc:.3f}")
    if "SQC_ICACHE_HITS" in v and "SQC_ICACHE_MISSES" in v:
        h, m = v["SQC_ICACHE_HITS"], v["SQC_ICACHE_MISSES"]
        print(f"{'icache miss rate':28s} {m / max(h + m, 1):.4f}")
    if cyc and "SQC_ICACHE_BUSY_CYCLES" in v:
        print(f"{'icache busy per SQC-cycle':28s} {v['SQC_ICACHE_BUSY_CYCLES'] / (NUM_CUS / 2) / cyc:.3f} (one SQC per 2 CUs)")
    for lvl, n in (("SQ_INST_LEVEL_LDS", "SQ_INSTS_LDS"), ("SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM_RD"),
                   ("SQ_IFETCH_LEVEL", "SQ_IFETCH")):
        if lvl in v and n in v and v[n]:
            print(f"{lvl + ' / ' + n:28s} {v[lvl] / v[n]:.1f} (avg latency, level units)")
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        print(f"HBM bytes (2*FETCH+WRITE)    {(2 * v['FETCH_SIZE'] + v['WRITE_SIZE']) * 1024:.4e}")


if __name__ == "__main__":
    main()
